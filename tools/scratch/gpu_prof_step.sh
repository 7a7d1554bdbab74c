#!/bin/bash
# kernel timeline of graph-replayed ConvNet steps (busy vs gaps) at the bench batch and at B=100
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
OUT=$R/gpurun_out/prof_step
mkdir -p $OUT
for B in ${BS:-32768 100}; do
  rm -rf /tmp/ps_$B
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ps_$B -o run -- python3 $R/bench.py --batch-per-rank $B --steps 30 --warmup 5 --comm-stats-steps 0 > $OUT/b$B.log 2>&1 || { tail -5 $OUT/b$B.log; exit 1; }
  cp $(find /tmp/ps_$B -name "*kernel_trace.csv" | head -1) $OUT/trace_b$B.csv
  cp $(find /tmp/ps_$B -name "*kernel_stats.csv" | head -1) $OUT/stats_b$B.csv
done
echo PROF_DONE
