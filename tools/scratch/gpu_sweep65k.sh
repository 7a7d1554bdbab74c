#!/bin/bash
# Role-split re-tune of the fused conv2/conv1 backward at the per-rank batch 65536 (two passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sw
b() { timeout -k 10 120 python bench.py --steps 60 --warmup 10 --comm-stats-steps 0 > gpurun_out/sw/x.log 2>&1 || exit 1; grep "^{" gpurun_out/sw/x.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])"; }
for r in 1 2; do for f in 0.58 0.60 0.62 0.64 0.66; do echo -n "c12frac $f "; RINGDP_C12_DGRAD_FRAC=$f b; done; done
