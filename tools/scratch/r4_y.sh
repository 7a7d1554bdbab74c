#!/bin/bash
# per-shape fp8 GEMM throughput (ViT-B/16 layer), CE-variant fusion tests, batched fp8 roll A/B
set -o pipefail
O=gpurun_out/r4y; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_convnet_model_gpu.py tests/test_nn_kernels_gpu.py -k "variants or batched_roll or fp8" > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --vit-fp8 > $O/gemm.log 2>&1 && \
for r in 1 0 1 0; do RINGDP_FP8_BATCH_ROLL=$r timeout -k 10 300 python -u bench.py --model vit_b_16 --dtype fp8 --steps 10 > $O/b_roll$r.json 2>>$O/b.err && cat $O/b_roll$r.json >> $O/ab.jsonl || exit 1; done && echo ALLDONE
tail -3 $O/tests.log; cat $O/gemm.log; cat $O/ab.jsonl | cut -c1-200
