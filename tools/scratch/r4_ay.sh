#!/bin/bash
# tile-row group size of the 256x256 kernels (final tree): 4 (default) vs 8
set -o pipefail
O=gpurun_out/r4ay; mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --model vit_b_16 $BARGS --steps 10 2>>$O/b.err | grep metric | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$tag', d['value'])" >> $O/ab.txt; }
for r in 1 2 3; do
  BARGS="" run "bf16 g4" X=0 || exit 1
  BARGS="" run "bf16 g8" RINGDP_BF16_GROUP_M=8 || exit 1
  BARGS="--dtype fp8" run "fp8 g4" X=0 || exit 1
  BARGS="--dtype fp8" run "fp8 g8" RINGDP_FP8_GROUP_M=8 || exit 1
done
cat $O/ab.txt
