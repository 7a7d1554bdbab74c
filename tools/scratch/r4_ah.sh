#!/bin/bash
# ViT-B/16 fp8 env sweep after the swizzle / MLPF8 changes: epilogue store form, tile groups, 256 round fill
set -o pipefail
O=gpurun_out/r4ah; mkdir -p $O
run() { env "$@" timeout -k 10 300 python -u bench.py --model vit_b_16 --dtype fp8 --steps 10 2>>$O/b.err | grep metric | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$*', d['value'])" >> $O/ab.txt; }
for r in 1 2; do
  run X=0 || exit 1
  run RINGDP_GEMM_WIDE_STORE=1 || exit 1
  run RINGDP_GEMM_WIDE_STORE=12 || exit 1
  run RINGDP_GEMM_STORE_CACHE=1 || exit 1
  run RINGDP_FP8_GROUP_M=8 || exit 1
  run RINGDP_FP8_GROUP_M=2 || exit 1
  run RINGDP_FP8_256_FILL=0.4 || exit 1
  run RINGDP_FP8_256_FILL=0.7 || exit 1
done
cat $O/ab.txt
