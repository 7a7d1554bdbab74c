# r3j: persistent 256x256 GEMM (tests, fixed-cost probe, ViT / ResNet-50 benches)
set -o pipefail
O=gpurun_out/r3j; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm256_gpu.py > $O/gemm_tests.log 2>&1; rc=$?; tail -3 $O/gemm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/gemm_epi_probe.py > $O/epi.jsonl 2>$O/epi.err || exit $?
cat $O/epi.jsonl
timeout -k 10 300 python tools/gemm_probe.py > $O/probe.jsonl 2>&1 || exit $?
cat $O/probe.jsonl | cut -c1-200
timeout -k 10 300 python bench.py --model vit_b_16 --steps 20 --warmup 5 --comm-stats-steps 0 > $O/b_vit.json 2>$O/b_vit.err || exit $?; grep -o '"value": [0-9.]*' $O/b_vit.json
timeout -k 10 300 python bench.py --model vit_b_16 --dtype fp8 --steps 20 --warmup 5 --comm-stats-steps 0 > $O/b_vit_fp8.json 2>$O/b_vit_fp8.err || exit $?; grep -o '"value": [0-9.]*' $O/b_vit_fp8.json
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 --comm-stats-steps 0 > $O/b_r50.json 2>$O/b_r50.err || exit $?; grep -o '"value": [0-9.]*' $O/b_r50.json
echo ALLDONE
