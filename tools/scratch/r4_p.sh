#!/bin/bash
# re-tune the backward role splits at B=65536 (set at B=32768 in round 3)
set -o pipefail
O=gpurun_out/r4p; mkdir -p $O; rm -f $O/times.jsonl
for f in 0.45 0.5 0.55; do
  for st in 0.05 0.1 0.15; do
    RINGDP_C3_DGRAD_FRAC=$f RINGDP_C3_STEAL=$st timeout -k 10 120 python tools/op_time.py conv3_fc_ce_bwd 65536 15 | sed "s/}/, \"frac\": $f, \"steal\": $st}/" >> $O/times.jsonl 2>>$O/t.err || exit 1
  done
done
for f in 0.58 0.64 0.7; do
  RINGDP_C12_DGRAD_FRAC=$f timeout -k 10 120 python tools/op_time.py conv12_bwd 65536 15 | sed "s/}/, \"c12frac\": $f}/" >> $O/times.jsonl 2>>$O/t.err || exit 1
done
cat $O/times.jsonl
echo ALLDONE
