#!/bin/bash
# fp8: all weights quantised in one launch per forward - tests + ViT fp8 bench A/B
set -o pipefail
O=gpurun_out/r4aq; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_nn_kernels_gpu.py -k "fp8" > $O/tests.log 2>&1 || { grep -E "Error|assert|FAIL" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for v in 0 1; do
  RINGDP_FP8_WQ_BATCH=$v timeout -k 10 300 python -u bench.py --model vit_b_16 --dtype fp8 --steps 10 2>>$O/b.err | grep metric | cut -c1-120 | sed "s/^/wq$v /" >> $O/ab.txt || exit 1
done; done
echo ALLDONE; cat $O/ab.txt
