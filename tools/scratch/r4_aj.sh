#!/bin/bash
# kernel table of the ViT-B/16 fp8 step after the e4m3 epilogues
set -o pipefail
O=gpurun_out/r4aj; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_vit16 -o run -- python3 $R/bench.py --model vit_b_16 --steps 10 > $R/$O/p.log 2>&1 || { tail -5 $R/$O/p.log; exit 1; }
cp $(find /tmp/p_vit16 -name "*kernel_stats.csv" | head -1) $R/$O/vit16_kernel_stats.csv
grep metric $R/$O/p.log | cut -c1-150; echo ALLDONE
