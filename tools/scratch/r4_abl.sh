#!/bin/bash
# conv3 backward ablations: same-box interleaved op timings of prebuilt variants (ab_so/<v>.so)
set -o pipefail
O=gpurun_out/r4abl; mkdir -p $O
for r in 1 2 3; do
  for v in base e p c epc; do
    for op in conv3_fc_bwd conv3_fc_bwd_w; do
      RINGDP_EXT_PATH=ab_so/$v.so timeout -k 10 120 python tools/op_time.py $op 65536 20 >> $O/times.jsonl 2>$O/$v.err || { echo "fail $v"; tail -3 $O/$v.err; exit 1; }
    done
  done
  tail -10 $O/times.jsonl
done
echo ALLDONE
