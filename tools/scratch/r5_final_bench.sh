#!/bin/bash
# round-5 evidence (2/2): 1-GPU benches of every model (incl. B=100 bf16 and fp32)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5final; mkdir -p $O
for m in "convnet" "convnet_fp32:--dtype fp32 --steps 5 --warmup 2" "resnet18:--model resnet18 --steps 20" "resnet50:--model resnet50 --steps 10" "vit:--model vit_b_16 --steps 10" "vit8:--model vit_b_16 --dtype fp8 --steps 10" "b100:--batch-per-rank 100 --steps 2000 --warmup 200" "b100fp32:--batch-per-rank 100 --dtype fp32 --steps 1000 --warmup 100"; do
  n=${m%%:*}; a=""; [ "$n" != "$m" ] && a=${m#*:}
  timeout -k 10 300 python -u bench.py $a > $O/b_$n.json 2>>$O/b.err || { echo "bench $n failed"; exit 1; }
  tail -1 $O/b_$n.json | cut -c1-150
done
echo ALLDONE
