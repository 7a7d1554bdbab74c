#!/bin/bash
# round 6: fused forward consumer k-step split sweep (phase 1 / 2 / 3 boundaries), headline bench A/B
set -o pipefail
O=gpurun_out/r6_ks
rm -rf $O; mkdir -p $O
B="timeout -k 10 120 python bench.py --steps 100 --warmup 20 --comm-stats-steps 0"
for r in 1 2; do
  $B > $O/base_$r.json 2>> $O/b.err || exit 1
  for v in ka3kb10 ka3kb11 ka5kb11 ka4kb12 ka5kb12 ka4kb10; do
    RINGDP_EXT_PATH=vtmp/$v.so $B > $O/${v}_$r.json 2>> $O/b.err || exit 1
  done
done
for f in $O/*.json; do python -c "import json,sys;d=json.loads(open('$f').read().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'])"; done
