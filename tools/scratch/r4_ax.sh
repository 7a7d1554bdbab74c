#!/bin/bash
# LayerNorm backward with the column sums compiled out unless requested: tests + ViT bench
set -o pipefail
O=gpurun_out/r4ax; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_nn_kernels_gpu.py tests/test_model_parity_gpu.py -k "layernorm or vit or fp8" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for d in bf16 fp8; do
  timeout -k 10 300 python -u bench.py --model vit_b_16 --dtype $d --steps 10 2>>$O/b.err | grep metric | cut -c1-120 | sed "s/^/$d /" >> $O/ab.txt || exit 1
done; done
echo ALLDONE; cat $O/ab.txt
