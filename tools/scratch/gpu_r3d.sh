# r3d: GEMM fixed-cost fit (8-B vs 16-B epilogue stores), GEMM tests, ViT bench, ConvNet headline
set -o pipefail
mkdir -p gpurun_out/r3d
timeout -k 10 300 python tools/gemm_fixed_cost.py > gpurun_out/r3d/fixed.jsonl 2>&1; echo fixed rc=$?
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm256_gpu.py tests/test_nn_kernels_gpu.py > gpurun_out/r3d/gemm_tests.log 2>&1; echo gemmtests rc=$?; tail -2 gpurun_out/r3d/gemm_tests.log
timeout -k 10 240 python bench.py --model vit_b_16 --steps 20 --warmup 5 --comm-stats-steps 0 > gpurun_out/r3d/bench_vit.json 2>>gpurun_out/r3d/bench.err; echo vit rc=$?; grep -o '"value": [0-9.]*' gpurun_out/r3d/bench_vit.json
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3d/bench_convnet.json 2>gpurun_out/r3d/bench_convnet.err; echo convnet rc=$?; grep -o '"value": [0-9.]*' gpurun_out/r3d/bench_convnet.json
timeout -k 10 200 python bench.py --batch-per-rank 100 --steps 200 --warmup 20 > gpurun_out/r3d/bench_b100.json 2>gpurun_out/r3d/bench_b100.err; echo b100 rc=$?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3d/bench_b100.json
