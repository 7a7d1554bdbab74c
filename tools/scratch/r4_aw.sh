#!/bin/bash
# kernel tables of the final ViT-B/16 bf16 and fp8 steps (stats csv only)
set -o pipefail
O=gpurun_out/r4aw; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for d in bf16 fp8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_$d -o run -- python3 $R/bench.py --model vit_b_16 --dtype $d --steps 10 > $R/$O/p_$d.log 2>&1 || { tail -5 $R/$O/p_$d.log; exit 1; }
  cp $(find /tmp/p_$d -name "*kernel_stats.csv" | head -1) $R/$O/vit_${d}_kernel_stats.csv
done
echo ALLDONE
