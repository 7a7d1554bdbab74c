#!/bin/bash
# fp8: LayerNorm forward writing the next linear's e4m3 input - tests + ViT fp8 bench A/B
set -o pipefail
O=gpurun_out/r4av; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_nn_kernels_gpu.py -k "fp8" > $O/tests.log 2>&1 || { grep -E "Error|assert|FAIL|tensor" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for v in 0 1; do
  RINGDP_FP8_LN_Q8=$v timeout -k 10 300 python -u bench.py --model vit_b_16 --dtype fp8 --steps 10 2>>$O/b.err | grep metric | cut -c1-120 | sed "s/^/lnq8_$v /" >> $O/ab.txt || exit 1
done; done
echo ALLDONE; cat $O/ab.txt
