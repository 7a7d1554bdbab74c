#!/bin/bash
set -o pipefail
O=gpurun_out/r4c3abl2; mkdir -p $O
for r in 1 2; do
  for v in base nocol nopool nomfma nowg nowg_nocol nowg_nopool; do
    RINGDP_EXT_PATH=ab_so/$v.so timeout -k 10 120 python tools/op_time.py conv3_fc_bwd 65536 15 >> $O/times.jsonl 2>>$O/t.err || { tail -3 $O/t.err; exit 1; }
  done
done
cat $O/times.jsonl
echo ALLDONE
