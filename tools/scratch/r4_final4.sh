#!/bin/bash
# round-4 final evidence: full GPU suite + smoke + 1-GPU benches of every model (incl. B=100 bf16 and fp32)
set -o pipefail
O=gpurun_out/r4final4; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/tests.log | head -20; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
for m in "convnet" "convnet_fp32:--dtype fp32 --steps 5 --warmup 2" "resnet18:--model resnet18 --steps 20" "resnet50:--model resnet50 --steps 10" "vit:--model vit_b_16 --steps 10" "vit8:--model vit_b_16 --dtype fp8 --steps 10" "b100:--batch-per-rank 100 --steps 2000 --warmup 200" "b100fp32:--batch-per-rank 100 --dtype fp32 --steps 1000 --warmup 100"; do
  n=${m%%:*}; a=""; [ "$n" != "$m" ] && a=${m#*:}
  timeout -k 10 300 python -u bench.py $a > $O/b_$n.json 2>>$O/b.err || { echo "bench $n failed"; exit 1; }
  grep metric $O/b_$n.json | cut -c1-150
done
echo ALLDONE
