#!/bin/bash
# round 6, first GPU pass: the new robustness tests + the ConvNet kernel/model suites, then the benches
set -o pipefail
mkdir -p gpurun_out/r6_t1
export PYTHONPATH=$PWD
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/r6_t1/b_convnet.json 2> gpurun_out/r6_t1/b_convnet.err && \
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --batch-per-rank 100 > gpurun_out/r6_t1/b_b100.json 2> gpurun_out/r6_t1/b_b100.err && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_convnet_kernels_gpu.py tests/test_convnet_model_gpu.py tests/test_watchdog_gpu.py tests/test_xgmi_gpu.py \
  > gpurun_out/r6_t1/tests.txt 2>&1
