#!/bin/bash
# round 6: fp32 conv3 data gradient in scatter form - numerics, then the fp32 bench A/B and a kernel table
set -o pipefail
O=gpurun_out/r6_t6
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_convnet_fp32_gpu.py > $O/tests.txt 2>&1 && \
timeout -k 10 300 python bench.py --dtype fp32 --steps 30 --warmup 5 --comm-stats-steps 0 > $O/b_fp32.json 2> $O/b_fp32.err && \
RINGDP_F32_DGRAD_SCATTER=0 timeout -k 10 300 python bench.py --dtype fp32 --steps 30 --warmup 5 --comm-stats-steps 0 > $O/b_fp32_off.json 2> $O/b_fp32_off.err && \
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fp32 -o run -- python3 bench.py --dtype fp32 --steps 20 --warmup 5 --comm-stats-steps 0 > $O/prof.log 2>&1
