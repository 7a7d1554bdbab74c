#!/bin/bash
# kernel tables of the final tree: ConvNet headline, ConvNet B=100 (bf16 / fp32), ViT-B/16 bf16
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_fprof; mkdir -p $O
for m in "convnet:--steps 20 --warmup 5" "b100:--batch-per-rank 100 --steps 200 --warmup 20" "b100fp32:--dtype fp32 --batch-per-rank 100 --steps 200 --warmup 20" "vit:--model vit_b_16 --steps 10 --warmup 3"; do
  n=${m%%:*}; a=${m#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$n -o run --output-format csv -- python3 bench.py $a --comm-stats-steps 0 > $O/p_$n.log 2>&1 || { tail -5 $O/p_$n.log; exit 1; }
  f=$(find $O/p_$n -name '*kernel_stats.csv' | head -1); python tools/prof_summary.py $f 30 > $O/k_$n.md; head -6 $O/k_$n.md
done
