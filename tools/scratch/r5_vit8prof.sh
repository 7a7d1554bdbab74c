#!/bin/bash
# ViT-B/16 fp8 and bf16 kernel tables (current tree)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_vit8prof; mkdir -p $O
for v in fp8 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$v -o run --output-format csv -- python3 bench.py --model vit_b_16 --dtype $v --steps 10 --warmup 3 --comm-stats-steps 0 > $O/p_$v.log 2>&1 || { tail -5 $O/p_$v.log; exit 1; }
  f=$(find $O/p_$v -name '*kernel_stats.csv' | head -1); python tools/prof_summary.py $f 45 > $O/k_$v.md
done
cat $O/k_fp8.md
