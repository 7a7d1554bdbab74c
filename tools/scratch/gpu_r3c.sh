# r3c: GEMM epilogue (loads hoisted) - probe, GEMM/NN kernel tests, extension-model benches
set -o pipefail
mkdir -p gpurun_out/r3c
timeout -k 10 300 python tools/gemm_probe.py > gpurun_out/r3c/probe2.jsonl 2>&1; echo probe rc=$?
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm256_gpu.py tests/test_nn_kernels_gpu.py > gpurun_out/r3c/gemm_tests.log 2>&1; echo gemmtests rc=$?; tail -3 gpurun_out/r3c/gemm_tests.log
for m in vit_b_16 resnet50 resnet18; do timeout -k 10 240 python bench.py --model $m --steps 20 --warmup 5 --comm-stats-steps 0 > gpurun_out/r3c/bench2_$m.json 2>>gpurun_out/r3c/bench.err; echo $m rc=$?; grep -o '"value": [0-9.]*' gpurun_out/r3c/bench2_$m.json; done
timeout -k 10 240 python bench.py --model vit_b_16 --dtype fp8 --steps 20 --warmup 5 --comm-stats-steps 0 > gpurun_out/r3c/bench2_vit_fp8.json 2>>gpurun_out/r3c/bench.err; echo fp8 rc=$?; grep -o '"value": [0-9.]*' gpurun_out/r3c/bench2_vit_fp8.json
