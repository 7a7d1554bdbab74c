#!/bin/bash
# fp32 B=100: forced data-gradient slice counts (every dgrad), step time + the conv3 / conv2 dgrad kernels
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_f32dgs; mkdir -p $O
for m in 2 3 4 6 8 12; do
  RINGDP_F32_DGRAD_SLICES=$m timeout -k 10 300 python -u bench.py --dtype fp32 --batch-per-rank 100 --steps 200 --warmup 20 --comm-stats-steps 0 > $O/b100_s$m.json 2>>$O/b.err || exit 1
  tail -1 $O/b100_s$m.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('B=100 slices=$m', d['value'], d['ms_per_step'])"
done
