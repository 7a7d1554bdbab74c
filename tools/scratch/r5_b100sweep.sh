#!/bin/bash
# B=100 bf16 step: conv3 weight-gradient slab size (RINGDP_C3_WMIN) and the dgrad share sweep
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_b100sweep; mkdir -p $O
B="timeout -k 10 200 python -u bench.py --batch-per-rank 100 --steps 3000 --warmup 300 --comm-stats-steps 0"
for r in 1 2; do
  for e in "X=0" "RINGDP_C3_WMIN=4" "RINGDP_C3_WMIN=8" "RINGDP_C3_WMIN=16" "RINGDP_C3_DGRAD_FRAC=0.35" "RINGDP_C3_DGRAD_FRAC=0.7"; do
    env $e $B > $O/b.json 2>>$O/b.err || exit 1
    echo "$e $(tail -1 $O/b.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"])')"
  done
done
