#!/bin/bash
# fp32 ConvNet (the reference's precision): B=65536 and B=100 benches + kernel tables
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_f32; mkdir -p $O
for B in 65536 100; do
  st=$([ $B = 100 ] && echo 200 || echo 10)
  timeout -k 10 300 python -u bench.py --dtype fp32 --batch-per-rank $B --steps $st --warmup 5 --comm-stats-steps 0 > $O/b_$B.json 2>>$O/b.err || exit 1
  tail -1 $O/b_$B.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('fp32 B=$B', d['value'], d['ms_per_step'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$B -o run --output-format csv -- python3 bench.py --dtype fp32 --batch-per-rank $B --steps $st --warmup 5 --comm-stats-steps 0 > $O/prof_$B.log 2>&1 || { tail -5 $O/prof_$B.log; exit 1; }
  f=$(find $O/prof_$B -name '*kernel_stats.csv' | head -1); python tools/prof_summary.py $f 40 > $O/k_$B.md; head -24 $O/k_$B.md
done
