#!/bin/bash
# round-5 closing evidence: the full GPU suite + smoke, then every bench config on the final tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5final5; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/tests.log | head -20; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for m in "convnet" "b100:--batch-per-rank 100 --steps 200 --warmup 20" "convnet_fp32:--dtype fp32" "b100fp32:--dtype fp32 --batch-per-rank 100 --steps 200 --warmup 20" \
         "vit:--model vit_b_16 --steps 10" "vit8:--model vit_b_16 --dtype fp8 --steps 10" "resnet50:--model resnet50 --steps 10" "resnet18:--model resnet18"; do
  n=${m%%:*}; a=""; [ "$n" != "$m" ] && a=${m#*:}
  timeout -k 10 300 python -u bench.py $a > $O/b_$n.json 2>>$O/b.err || { echo "bench $n failed"; exit 1; }
  tail -1 $O/b_$n.json | cut -c1-150
done
