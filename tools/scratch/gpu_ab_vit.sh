#!/bin/bash
# ViT kernel experiments: fp8 quantise-transpose tile (qt128 vs qt64), attention P store (default / 16-B
# paired / none), numerics of each variant, and the fp8 ViT step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S=ringdp/_C.cpython-310-x86_64-linux-gnu.so
T="python -u -m pytest tests/test_nn_kernels_gpu.py -k fp8_or_vit_or_attention -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 python -u -m pytest tests/test_nn_kernels_gpu.py -k "fp8 or vit or attention" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_qt.log 2>&1; tail -1 gpurun_out/t_qt.log
cp abv/p16.so $S && timeout -k 10 300 python -u -m pytest tests/test_nn_kernels_gpu.py -k "vit or attention" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_p16.log 2>&1; echo -n "p16 tests: "; tail -1 gpurun_out/t_p16.log
cp abv/qt128.so $S
AB_CMD="python tools/fp8q_bench.py" bash tools/gpu_ab_so.sh qt128 qt64 || exit 1
AB_CMD="python tools/attn_bench.py" bash tools/gpu_ab_so.sh qt128 p16 nop || exit 1
BENCH_ARGS="--model vit_b_16 --dtype fp8 --steps 20 --warmup 3" bash tools/gpu_ab_so.sh qt128 qt64 p16 || exit 1
echo ALLDONE
