#!/bin/bash
# headline: images per fc1-backward workgroup at B=65536 (512 / 1024 / 2048 workgroups)
set -o pipefail
O=gpurun_out/r4ar; mkdir -p $O
for r in 1 2; do for v in 128 64 32; do
  RINGDP_CN_FC_IMGS=$v timeout -k 10 300 python -u bench.py 2>>$O/b.err | grep metric | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('fc_imgs=$v', d['value'], d['ms_per_step'])" >> $O/ab.txt || exit 1
done; done
cat $O/ab.txt
