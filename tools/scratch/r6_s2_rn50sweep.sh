#!/bin/bash
# round 6 (session 2): ResNet-50 GEMM routing / split knobs
set -o pipefail
O=gpurun_out/r6_s2_rn50sweep
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
B="timeout -k 10 180 python bench.py --model resnet50 --steps 30 --comm-stats-steps 0"
run() { local n=$1; shift; env "$@" $B > $O/$n.json 2>> $O/b.err || exit 1; }
for r in 1 2; do
  run base_$r X=1
  run f40_$r RINGDP_BF16_256_FILL=0.40
  run f70_$r RINGDP_BF16_256_FILL=0.70
  run cw1024_$r RINGDP_CONV_SPLIT_WGS=1024
  run ww1024_$r RINGDP_WGRAD_SPLIT_WGS=1024
  run t128_$r RINGDP_BF16_TILE=128
done
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
echo DONE >> $O/summary.txt
