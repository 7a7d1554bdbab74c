#!/bin/bash
# fp32 B=100: weight-gradient slice depth sweep (RINGDP_F32_WGRAD_MIN_K), then B=65536 at the smallest
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_f32wgs; mkdir -p $O
for d in 1024 512 256 128; do
  RINGDP_F32_WGRAD_MIN_K=$d timeout -k 10 300 python -u bench.py --dtype fp32 --batch-per-rank 100 --steps 200 --warmup 20 --comm-stats-steps 0 > $O/b100_d$d.json 2>>$O/b.err || exit 1
  tail -1 $O/b100_d$d.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('B=100 min_k=$d', d['value'], d['ms_per_step'])"
done
for d in 1024 256; do
  RINGDP_F32_WGRAD_MIN_K=$d timeout -k 10 300 python -u bench.py --dtype fp32 --comm-stats-steps 0 > $O/b65536_d$d.json 2>>$O/b.err || exit 1
  tail -1 $O/b65536_d$d.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('B=65536 min_k=$d', d['value'], d['ms_per_step'])"
done
