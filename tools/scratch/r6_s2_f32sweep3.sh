#!/bin/bash
# round 6 (session 2): fp32 B=100 forward / data-gradient k slices on the 320-deep weight-gradient default
set -o pipefail
O=gpurun_out/r6_s2_f32sweep3
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
B="timeout -k 10 120 python bench.py --batch-per-rank 100 --dtype fp32 --steps 2000 --warmup 200 --comm-stats-steps 0"
run() { local n=$1; shift; env "$@" $B > $O/$n.json 2>> $O/b.err || exit 1; }
for r in 1 2; do
  run base_$r X=1
  run fs1_$r RINGDP_F32_FWD_SLICES=1
  run fs2_$r RINGDP_F32_FWD_SLICES=2
  run fs3_$r RINGDP_F32_FWD_SLICES=3
  run fs6_$r RINGDP_F32_FWD_SLICES=6
  run ds4_$r RINGDP_F32_DGRAD_SLICES=4
  run ds6_$r RINGDP_F32_DGRAD_SLICES=6
  run ds10_$r RINGDP_F32_DGRAD_SLICES=10
done
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
echo DONE >> $O/summary.txt
