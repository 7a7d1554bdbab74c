#!/bin/bash
# round 6: fp32 conv2 fwd prefetch
set -o pipefail
O=gpurun_out/r6_t13
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_convnet_fp32_gpu.py -k "conv2_pool or matches_aten" > $O/tests.txt 2>&1 && \
timeout -k 10 300 python bench.py --dtype fp32 --steps 30 --warmup 5 --comm-stats-steps 0 > $O/b_fp32.json 2> $O/b_fp32.err && \
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fp32 -o run -- python3 bench.py --dtype fp32 --steps 20 --warmup 5 --comm-stats-steps 0 > $O/prof.log 2>&1
