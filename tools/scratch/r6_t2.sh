#!/bin/bash
# round 6: the pool2 producer/consumer split sweep, kernel tables at B=65536 / B=100, remaining GPU tests
set -o pipefail
O=gpurun_out/r6_t2
mkdir -p $O
export PYTHONPATH=$PWD
for p2 in 400 512 560 640 720; do
  RINGDP_FF_P2=$p2 timeout -k 10 120 python bench.py --steps 200 --warmup 20 --comm-stats-steps 0 > $O/p2_$p2.json 2> $O/p2_$p2.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b65536 -o run -- python3 bench.py --steps 100 --warmup 20 --comm-stats-steps 0 > $O/prof_b65536.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b100 -o run -- python3 bench.py --steps 2000 --warmup 50 --batch-per-rank 100 --comm-stats-steps 0 > $O/prof_b100.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -v --timeout 240 --timeout-method thread \
  tests/test_watchdog_gpu.py tests/test_xgmi_gpu.py > $O/tests.txt 2>&1
