#!/bin/bash
# round 6 (session 2): ResNet-18 split-K count sweep (conv forward / data-gradient GEMM splits, weight-gradient splits)
set -o pipefail
O=gpurun_out/r6_s2_rnsplit
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
B="timeout -k 10 120 python bench.py --model resnet18 --steps 200 --comm-stats-steps 0"
run() { local n=$1; shift; env "$@" $B > $O/$n.json 2>> $O/b.err || exit 1; }
for r in 1 2; do
  run base_$r X=1
  run cw256_$r RINGDP_CONV_SPLIT_WGS=256
  run cw1024_$r RINGDP_CONV_SPLIT_WGS=1024
  run ck2_$r RINGDP_CONV_SPLIT_MINKT=2
  run ck8_$r RINGDP_CONV_SPLIT_MINKT=8
  run ww256_$r RINGDP_WGRAD_SPLIT_WGS=256
  run ww1024_$r RINGDP_WGRAD_SPLIT_WGS=1024
  run wk2_$r RINGDP_WGRAD_SPLIT_MINKT=2
  run wk8_$r RINGDP_WGRAD_SPLIT_MINKT=8
done
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
echo DONE >> $O/summary.txt
