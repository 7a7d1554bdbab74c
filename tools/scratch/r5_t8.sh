#!/bin/bash
# same-box A/B (abv/base.so vs tree) + PMC of the tree's backward kernels + rocprof table
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-.}
bash $R/tools/scratch/r5_ab.sh r5_t8 "conv3_fc_ce_bwd conv12_bwd" convnet || exit 1
bash $R/tools/scratch/r5_pmc2.sh r5_t8/pmc 65536 conv3_fc_ce_bwd > /dev/null && \
bash $R/tools/scratch/r5_pmc2.sh r5_t8/pmc 65536 conv12_bwd > /dev/null && \
bash $R/tools/scratch/r5_pmc2.sh r5_t8/pmc 65536 fwd_fused > /dev/null || exit 1
cd $R
O=gpurun_out/r5_t8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); python tools/prof_summary.py $f 14 > $O/prof_kernels.md; cat $O/prof_kernels.md
