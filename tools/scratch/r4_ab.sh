#!/bin/bash
# e4m3-output GEMM epilogue (MLPF8): tests, per-op timing, ViT fp8 bench A/B
set -o pipefail
O=gpurun_out/r4ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_nn_kernels_gpu.py -k "fp8 or quant_out" > $O/tests.log 2>&1 || { grep -E "Error|error|assert|FAIL" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|unfused" $O/tests.log | tail -20
for r in 1 2; do for v in 0 1; do
  RINGDP_FP8_MLP_FUSED=$v timeout -k 10 300 python -u bench.py --model vit_b_16 --dtype fp8 --steps 10 2>>$O/b.err | grep metric | sed "s/^/fused$v /" >> $O/ab.txt || exit 1
done; done
echo ALLDONE; cut -c1-130 $O/ab.txt
