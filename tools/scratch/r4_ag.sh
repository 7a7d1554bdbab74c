#!/bin/bash
# B=100 bf16: images per weight-gradient slab (fewer slabs = shorter reduction, fewer backward workgroups)
set -o pipefail
O=gpurun_out/r4ag; mkdir -p $O
for r in 1 2; do for w in "2 2" "4 4" "8 8" "4 2" "2 4"; do set -- $w
  RINGDP_C3_WMIN=$1 RINGDP_C12_WMIN=$2 timeout -k 10 200 python -u bench.py --batch-per-rank 100 --steps 2000 --warmup 200 2>>$O/b.err | grep metric | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('c3=$1 c12=$2', d['value'], d['ms_per_step'])" >> $O/ab.txt || exit 1
done; done
cat $O/ab.txt
