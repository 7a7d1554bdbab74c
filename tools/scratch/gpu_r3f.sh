# r3f: session re-entry evidence: full GPU suite, every bench config, kernel table for ViT/ResNet-50
set -o pipefail
O=gpurun_out/r3f; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 $O/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py > $O/b_convnet.json 2>$O/b_convnet.err || exit $?; cat $O/b_convnet.json | cut -c1-300
timeout -k 10 200 python bench.py --batch-per-rank 100 --steps 300 --warmup 20 > $O/b_b100.json 2>$O/b_b100.err || exit $?; grep -o '"ms_per_step": [0-9.]*' $O/b_b100.json
for m in resnet18 resnet50 vit_b_16; do timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > $O/b_$m.json 2>$O/b_$m.err || exit $?; echo $m; grep -o '"value": [0-9.]*' $O/b_$m.json; done
timeout -k 10 300 python bench.py --model vit_b_16 --dtype fp8 --steps 20 --warmup 5 > $O/b_vit_fp8.json 2>$O/b_vit_fp8.err || exit $?; grep -o '"value": [0-9.]*' $O/b_vit_fp8.json
timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 > $O/b_fp32.json 2>$O/b_fp32.err || exit $?; grep -o '"value": [0-9.]*' $O/b_fp32.json
cd /tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vit -o run --output-format csv -- python3 bench.py --model vit_b_16 --steps 5 --warmup 2 --no-graph --comm-stats-steps 0 > $O/prof_vit.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vit_fp8 -o run --output-format csv -- python3 bench.py --model vit_b_16 --dtype fp8 --steps 5 --warmup 2 --no-graph --comm-stats-steps 0 > $O/prof_vit_fp8.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r50 -o run --output-format csv -- python3 bench.py --model resnet50 --steps 5 --warmup 2 --no-graph --comm-stats-steps 0 > $O/prof_r50.log 2>&1 || exit $?
echo ALLDONE
