#!/bin/bash
# round 6 (session 2): bf16 B=100 backward role split re-sweep on the whole-network node
set -o pipefail
O=gpurun_out/r6_s2_b100sweep
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
B="timeout -k 10 120 python bench.py --batch-per-rank 100 --steps 2000 --warmup 200 --comm-stats-steps 0"
run() { local n=$1; shift; env "$@" $B > $O/$n.json 2>> $O/b.err || exit 1; }
for r in 1 2; do
  run base_$r X=1
  run c3w1_$r RINGDP_C3_WMIN=1
  run c3w4_$r RINGDP_C3_WMIN=4
  run c12w1_$r RINGDP_C12_WMIN=1
  run c12w4_$r RINGDP_C12_WMIN=4
  run c3f3_$r RINGDP_C3_DGRAD_FRAC=0.3
  run c12f3_$r RINGDP_C12_DGRAD_FRAC=0.3
done
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
echo DONE >> $O/summary.txt
