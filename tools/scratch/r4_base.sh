#!/bin/bash
# round-4 baseline: ConvNet bench, kernel trace, PMC of the two backward kernels at B=65536
set -o pipefail
O=gpurun_out/r4base; mkdir -p $O
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b_convnet.json 2>$O/b_convnet.err || exit $?; echo convnet $(grep -o '"value": [0-9.]*' $O/b_convnet.json)
R=$PWD
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 30 --warmup 5 --comm-stats-steps 0 > $R/$O/prof.log 2>&1) || exit $?
python3 tools/prof_summary.py $(find $O/prof -name "*kernel_stats.csv" | head -1) > $O/prof_kernels.md 2>&1; head -20 $O/prof_kernels.md
for op in conv3_fc_bwd conv12_bwd; do bash tools/pmc_op.sh $op 65536 r4base || exit 1; done
echo ALLDONE
