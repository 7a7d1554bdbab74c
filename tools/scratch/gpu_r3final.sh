# round-3 evidence: full GPU suite, every bench config (default ConvNet, reference batch, fp32, ResNet-18/50, ViT bf16/fp8),
# fp32 ConvNet kernel trace
set -o pipefail
O=gpurun_out/${RUN:-r3final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py > $O/b_convnet.json 2>$O/b_convnet.err || exit $?; echo convnet $(grep -o '"value": [0-9.]*' $O/b_convnet.json)
timeout -k 10 200 python bench.py --batch-per-rank 100 --steps 200 --warmup 20 > $O/b_convnet_b100.json 2>$O/b_convnet_b100.err || exit $?; echo b100 $(grep -o '"ms_per_step": [0-9.]*' $O/b_convnet_b100.json)
timeout -k 10 200 python bench.py --dtype fp32 --steps 10 --warmup 3 > $O/b_convnet_fp32.json 2>$O/b_convnet_fp32.err || exit $?; echo fp32 $(grep -o '"value": [0-9.]*' $O/b_convnet_fp32.json)
for m in resnet18 resnet50 vit_b_16; do timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --comm-stats-steps 0 > $O/b_$m.json 2>$O/b_$m.err || exit $?; echo $m $(grep -o '"value": [0-9.]*' $O/b_$m.json); done
timeout -k 10 300 python bench.py --model vit_b_16 --dtype fp8 --steps 20 --warmup 5 --comm-stats-steps 0 > $O/b_vit_fp8.json 2>$O/b_vit_fp8.err || exit $?; echo vit_fp8 $(grep -o '"value": [0-9.]*' $O/b_vit_fp8.json)
cd /tmp; cd - >/dev/null; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_f32 -o run --output-format csv -- python3 bench.py --dtype fp32 --steps 3 --warmup 1 --comm-stats-steps 0 > $O/prof_f32.log 2>&1 || exit $?
echo ALLDONE
