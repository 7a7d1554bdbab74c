#!/bin/bash
# round 6: fp32 conv3 wgrad natural layout + prefetch
set -o pipefail
O=gpurun_out/r6_t12
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_convnet_fp32_gpu.py -k "matches_aten or convergence" > $O/tests.txt 2>&1
