#!/bin/bash
# round 6 final: the whole GPU suite (one process), smoke, every model's bench, kernel tables of the ConvNet configs
# and ResNet-18
set -o pipefail
O=gpurun_out/r6_final
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
for m in "convnet" "convnet_fp32:--dtype fp32 --steps 30 --warmup 5" "b100:--batch-per-rank 100 --steps 2000 --warmup 200" "b100fp32:--batch-per-rank 100 --dtype fp32 --steps 2000 --warmup 200" "resnet18:--model resnet18 --steps 200" "resnet50:--model resnet50 --steps 20" "vit:--model vit_b_16 --steps 20" "vit8:--model vit_b_16 --dtype fp8 --steps 20"; do
  n=${m%%:*}; a=""; [ "$n" != "$m" ] && a=${m#*:}
  timeout -k 10 300 python -u bench.py $a --comm-stats-steps 20 > $O/b_$n.json 2>>$O/b.err || { echo "bench $n failed"; exit 1; }
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for m in "convnet:--steps 200" "b100:--batch-per-rank 100 --steps 1000" "b100fp32:--batch-per-rank 100 --dtype fp32 --steps 500" "convnet_fp32:--dtype fp32 --steps 20 --warmup 5" "resnet18:--model resnet18 --steps 100"; do
  n=${m%%:*}; a=${m#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run -- python3 bench.py $a --comm-stats-steps 0 > $O/prof_$n.log 2>&1 || { echo "prof $n failed"; exit 1; }
done
for f in $O/b_*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
echo ALLDONE
