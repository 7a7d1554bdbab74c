#!/bin/bash
# headline: fc1 backward inside the conv3 backward launch at B=65536 too (compact gradient computed in place)?
set -o pipefail
O=gpurun_out/r4am; mkdir -p $O
for r in 1 2; do for v in 0 1; do
  RINGDP_CN_DA3_INPLACE=$v timeout -k 10 300 python -u bench.py 2>>$O/b.err | grep metric | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('da3_inplace=$v', d['value'], d['ms_per_step'])" >> $O/ab.txt || exit 1
done; done
cat $O/ab.txt
