#!/bin/bash
# round-fill thresholds of the 256x256 kernels after the round-4 changes (ViT bf16 / fp8)
set -o pipefail
O=gpurun_out/r4at; mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --model vit_b_16 $BARGS --steps 10 2>>$O/b.err | grep metric | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$tag', d['value'])" >> $O/ab.txt; }
for r in 1 2; do
  BARGS="" run "bf16 fill=0.55" X=0 || exit 1
  BARGS="" run "bf16 fill=0.45" RINGDP_BF16_256_FILL=0.45 || exit 1
  BARGS="" run "bf16 fill=0.65" RINGDP_BF16_256_FILL=0.65 || exit 1
  BARGS="--dtype fp8" run "fp8 fill=0.55" X=0 || exit 1
  BARGS="--dtype fp8" run "fp8 fill=0.40" RINGDP_FP8_256_FILL=0.40 || exit 1
done
cat $O/ab.txt
