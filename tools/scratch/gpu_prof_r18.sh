#!/bin/bash
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
OUT=$R/gpurun_out/prof_r18
mkdir -p $OUT
rm -rf /tmp/pr18
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d /tmp/pr18 -o run -- python3 $R/bench.py --model resnet18 --steps 30 --warmup 5 --comm-stats-steps 0 ${EXTRA:-} > $OUT/log 2>&1 || { tail -5 $OUT/log; exit 1; }
cp $(find /tmp/pr18 -name "*kernel_trace.csv" | head -1) $OUT/trace.csv
echo PROF_DONE
