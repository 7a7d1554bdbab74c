#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sweep
mkdir -p $OUT
for f in 0.45 0.5 0.55 0.6 0.65; do
  timeout -k 10 120 env RINGDP_C2_DGRAD_FRAC=$f RINGDP_C3_DGRAD_FRAC=${C3:-0.55} python tools/kbench.py 32768 > $OUT/c2_$f.log 2>&1 || exit 1
  echo "c2 $f $(grep -o '"conv2_bwd": {"us": [0-9.]*' $OUT/c2_$f.log)"
done
for f in 0.5 0.53 0.57 0.6; do
  timeout -k 10 120 env RINGDP_C3_DGRAD_FRAC=$f python tools/kbench.py 32768 > $OUT/c3_$f.log 2>&1 || exit 1
  echo "c3 $f $(grep -o '"conv3_fc_bwd": {"us": [0-9.]*' $OUT/c3_$f.log)"
done
