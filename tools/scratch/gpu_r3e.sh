# r3e: GEMM epilogue store modes (0 8-B, 1 lane-exchange 16-B, 2 LDS-staged rows, 3 discard)
set -o pipefail
mkdir -p gpurun_out/r3e
timeout -k 10 300 python tools/gemm_fixed_cost.py > gpurun_out/r3e/fixed.jsonl 2>&1; echo fixed rc=$?
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm256_gpu.py > gpurun_out/r3e/gemm_tests.log 2>&1; echo gemmtests rc=$?; tail -2 gpurun_out/r3e/gemm_tests.log
