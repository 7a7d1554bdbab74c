#!/bin/bash
# round-5 evidence refresh after the ViT epilogue/cast changes: ViT bf16 + fp8, ResNet-50, ConvNet headline
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5final2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "vit or gemm or fp8 or resnet" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
for m in "convnet" "vit:--model vit_b_16 --steps 10" "vit8:--model vit_b_16 --dtype fp8 --steps 10" "resnet50:--model resnet50 --steps 10"; do
  n=${m%%:*}; a=""; [ "$n" != "$m" ] && a=${m#*:}
  timeout -k 10 300 python -u bench.py $a > $O/b_$n.json 2>>$O/b.err || { echo "bench $n failed"; exit 1; }
  tail -1 $O/b_$n.json | cut -c1-150
done
