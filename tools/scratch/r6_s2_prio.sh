#!/bin/bash
# round 6 (session 2): fused forward A/B - wave issue priority per phase (RINGDP_FF_PRIO variants in vtmp/)
set -o pipefail
O=gpurun_out/r6_s2_prio
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
B="timeout -k 10 120 python bench.py --steps 200 --warmup 20 --comm-stats-steps 0"
for r in 1 2; do
  $B > $O/base_$r.json 2>> $O/b.err || exit 1
  for v in prio1 prio2 prio3 bprio fbprio; do
    RINGDP_EXT_PATH=vtmp/$v.so $B > $O/${v}_$r.json 2>> $O/b.err || exit 1
  done
done
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
