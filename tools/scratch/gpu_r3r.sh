# r3r: bf16-oracle parity + B=4096 trajectory tests; fp8 256-kernel routing; GEMM tests; ViT fp8 bench
set -o pipefail
O=gpurun_out/r3r; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_convnet_model_gpu.py > $O/tests.log 2>&1; rc=$?; grep -E "passed|failed|max \||\{'conv" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model vit_b_16 --dtype fp8 --steps 20 --warmup 5 --comm-stats-steps 0 > $O/b_vit_fp8.json 2>$O/b_vit_fp8.err || exit $?; grep -o '"value": [0-9.]*' $O/b_vit_fp8.json
echo ALLDONE
