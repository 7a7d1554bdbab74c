#!/bin/bash
# round 6 (session 2): BN partial-row count sweep (ResNet-50, ResNet-18)
set -o pipefail
O=gpurun_out/r6_s2_bnparts
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
B="timeout -k 10 180 python bench.py --model resnet50 --steps 30 --comm-stats-steps 0"
run() { local n=$1; shift; env "$@" $B > $O/$n.json 2>> $O/b.err || exit 1; }
for r in 1 2; do
  run base_$r X=1
  run mp256_$r RINGDP_BN_MAX_PARTS=256
  run mp512_$r RINGDP_BN_MAX_PARTS=512
  run mp2048_$r RINGDP_BN_MAX_PARTS=2048
  run mr128_$r RINGDP_BN_MIN_ROWS=128
done
B="timeout -k 10 120 python bench.py --model resnet18 --steps 200 --comm-stats-steps 0"
for r in 1 2; do
  run rn18_base_$r X=1
  run rn18_mr128_$r RINGDP_BN_MIN_ROWS=128
  run rn18_mr32_$r RINGDP_BN_MIN_ROWS=32
done
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
echo DONE >> $O/summary.txt
