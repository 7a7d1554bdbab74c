#!/bin/bash
# round-5 baseline: headline bench + rocprofv3 kernel stats of the B=65536 ConvNet step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5base; mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/b_convnet.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
cat $O/b_convnet.json | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); python tools/prof_summary.py $f 12 > $O/prof_kernels.md; cat $O/prof_kernels.md
