# r3p: generic GEMM epilogue on uniform flags + branch-free erf: full GPU suite, every bench config
set -o pipefail
O=gpurun_out/r3p; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -le 1 ] || exit $rc; [ $rc -eq 0 ] || exit 1
for m in vit_b_16 resnet50 resnet18; do timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --comm-stats-steps 0 > $O/b_$m.json 2>$O/b_$m.err || exit $?; echo $m; grep -o '"value": [0-9.]*' $O/b_$m.json; done
timeout -k 10 300 python bench.py --model vit_b_16 --dtype fp8 --steps 20 --warmup 5 --comm-stats-steps 0 > $O/b_vit_fp8.json 2>$O/b_vit_fp8.err || exit $?; grep -o '"value": [0-9.]*' $O/b_vit_fp8.json
timeout -k 10 200 python bench.py > $O/b_convnet.json 2>$O/b_convnet.err || exit $?; grep -o '"value": [0-9.]*' $O/b_convnet.json
cd /tmp; cd - >/dev/null; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vit -o run --output-format csv -- python3 bench.py --model vit_b_16 --steps 5 --warmup 2 --no-graph --comm-stats-steps 0 > $O/prof_vit.log 2>&1 || exit $?
echo ALLDONE
