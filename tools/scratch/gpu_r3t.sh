# r3t: ConvNet model tests (bf16 oracle) on the kept kernels; fp8 ViT bench; ConvNet step kernel table
set -o pipefail
O=gpurun_out/r3t; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_convnet_model_gpu.py tests/test_convnet_kernels_gpu.py > $O/tests.log 2>&1; rc=$?; grep -E "passed|failed|^l2" $O/tests.log | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model vit_b_16 --dtype fp8 --steps 20 --warmup 5 --comm-stats-steps 0 > $O/b_vit_fp8.json 2>$O/b_vit_fp8.err || exit $?; grep -o '"value": [0-9.]*' $O/b_vit_fp8.json
cd /tmp; cd - >/dev/null; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cn -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --comm-stats-steps 0 > $O/prof_cn.log 2>&1 || exit $?
echo ALLDONE
