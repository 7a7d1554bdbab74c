#!/bin/bash
# round 6 (session 2): headline (bf16, B=65536) backward role split re-sweep on the final tree
set -o pipefail
O=gpurun_out/r6_s2_hlsweep5
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
B="timeout -k 10 120 python bench.py --steps 100 --warmup 10 --comm-stats-steps 0"
run() { local n=$1; shift; env "$@" $B > $O/$n.json 2>> $O/b.err || exit 1; }
for r in 1 2 3; do
  run base_$r X=1
  run c12f63_$r RINGDP_C12_DGRAD_FRAC=0.63
  run c3f53_$r RINGDP_C3_DGRAD_FRAC=0.53
done
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
echo DONE >> $O/summary.txt
