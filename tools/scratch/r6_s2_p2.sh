#!/bin/bash
# round 6 (session 2): pool2 producer/consumer item split re-sweep after the pool2 rewrite (RINGDP_FF_P2)
set -o pipefail
O=gpurun_out/r6_s2_p2
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
B="timeout -k 10 120 python bench.py --steps 100 --warmup 20 --comm-stats-steps 0"
for r in 1 2; do
  for v in 560 800 768 704 640; do
    RINGDP_FF_P2=$v $B > $O/p2_${v}_$r.json 2>> $O/b.err || exit 1
  done
done
for f in $O/*.json; do python -c "import json,sys;d=json.loads(open('$f').read().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
