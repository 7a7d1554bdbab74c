#!/bin/bash
# ViT bf16 kernel tables with the 2-WG GEMM off / on (RINGDP_GEMM_2WG=0 / 2)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_2wgp; mkdir -p $O
for m in 0 2; do
  RINGDP_GEMM_2WG=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- python3 bench.py --model vit_b_16 --steps 10 --warmup 3 --comm-stats-steps 0 > $O/prof_$m.log 2>&1 || { tail -5 $O/prof_$m.log; exit 1; }
  f=$(find $O/prof_$m -name '*kernel_stats.csv' | head -1); python tools/prof_summary.py $f 40 > $O/k_$m.md; grep -E "gemm" $O/k_$m.md
done
