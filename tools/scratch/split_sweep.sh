#!/bin/bash
# Sweep the dgrad/wgrad CU split of the role-fused ConvNet backward launches.
# usage: tools/split_sweep.sh [B] ; prints "<layer> <frac> <us>" per point.
B=${1:-16384}
for f in ${C3_FRACS:-0.5 0.56 0.62 0.68 0.74 0.8}; do
  us=$(RINGDP_C3_DGRAD_FRAC=$f timeout -k 10 120 python tools/kbench.py $B | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['conv3_fc_bwd']['us'])") || exit 1
  echo "C3 $f $us"
done
for f in ${C2_FRACS:-0.44 0.5 0.56 0.62 0.68 0.74}; do
  us=$(RINGDP_C2_DGRAD_FRAC=$f timeout -k 10 120 python tools/kbench.py $B | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['conv2_bwd']['us'])") || exit 1
  echo "C2 $f $us"
done
