#!/bin/bash
# attention with P recomputed in the backward: tests, ViT bf16 / fp8 bench A/B
set -o pipefail
O=gpurun_out/r4ai; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_nn_kernels_gpu.py tests/test_model_parity_gpu.py -k "attention or attn or vit" > $O/tests.log 2>&1 || { grep -E "Error|error|assert|FAIL" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
grep -cE "PASSED" $O/tests.log; tail -2 $O/tests.log
for r in 1 2; do for v in 0 1; do
  RINGDP_ATTN_RECOMPUTE=$v timeout -k 10 300 python -u bench.py --model vit_b_16 --steps 10 2>>$O/b.err | grep metric | sed "s/^/bf16 rec$v /" >> $O/ab.txt || exit 1
  RINGDP_ATTN_RECOMPUTE=$v timeout -k 10 300 python -u bench.py --model vit_b_16 --dtype fp8 --steps 10 2>>$O/b.err | grep metric | sed "s/^/fp8 rec$v /" >> $O/ab.txt || exit 1
done; done
echo ALLDONE; cut -c1-120 $O/ab.txt
