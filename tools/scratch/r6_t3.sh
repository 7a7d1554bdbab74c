#!/bin/bash
# round 6: watchdog + xgmi suites after the test fixes, and the B=100 bench with the whole-network node
set -o pipefail
O=gpurun_out/r6_t3
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --batch-per-rank 100 > $O/b_b100.json 2> $O/b_b100.err && \
timeout -k 10 900 python -u -m pytest -v --timeout 240 --timeout-method thread \
  tests/test_watchdog_gpu.py tests/test_xgmi_gpu.py > $O/tests.txt 2>&1
