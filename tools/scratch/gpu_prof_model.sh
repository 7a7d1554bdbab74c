#!/bin/bash
# kernel trace of graph-replayed steps of one bench model: bash tools/gpu_prof_model.sh <model> [extra bench args]
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
M=$1; shift
OUT=$R/gpurun_out/prof_$M
mkdir -p $OUT
rm -rf /tmp/pm_$M
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/pm_$M -o run -- python3 $R/bench.py --model $M --steps ${STEPS:-5} --warmup 3 --comm-stats-steps 0 "$@" > $OUT/log 2>&1 || { tail -5 $OUT/log; exit 1; }
cp $(find /tmp/pm_$M -name "*kernel_trace.csv" | head -1) $OUT/trace.csv
echo PROF_DONE
