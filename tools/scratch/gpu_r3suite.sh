# full GPU suite on the final round-3 tree + ViT bench
set -o pipefail
O=gpurun_out/${RUN:-r3suite}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --model vit_b_16 --steps 20 --warmup 5 --comm-stats-steps 0 > $O/b_vit_b_16.json 2>$O/b_vit.err || exit $?; echo vit $(grep -o '"value": [0-9.]*' $O/b_vit_b_16.json)
timeout -k 10 200 python bench.py > $O/b_convnet.json 2>$O/b_convnet.err || exit $?; echo convnet $(grep -o '"value": [0-9.]*' $O/b_convnet.json)
echo ALLDONE
