#!/bin/bash
# bf16 GEMM epilogue column sums (MLPF fc1 bias gradient): tests + ViT bf16 bench
set -o pipefail
O=gpurun_out/r4as; mkdir -p $O
RINGDP_LN_COLSUM=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_nn_kernels_gpu.py tests/test_gemm256_gpu.py tests/test_model_parity_gpu.py -k "colsum or layernorm or vit or mlp or attention" > $O/tests.log 2>&1 || { grep -E "Error|assert|FAIL" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 0 1; do RINGDP_LN_COLSUM=$v timeout -k 10 300 python -u bench.py --model vit_b_16 --steps 10 2>>$O/b.err | grep metric | cut -c1-130 | sed "s/^/lncs$v /" >> $O/ab.txt || exit 1; done
done
echo ALLDONE; cat $O/ab.txt
