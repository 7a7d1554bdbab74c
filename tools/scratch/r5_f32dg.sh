#!/bin/bash
# fp32 split-K data gradient at small batches: fp32 tests, B=100 / B=65536 benches with it off (1) / auto, B=100 table
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_f32w1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "f32 or fp32" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
for r in 1 2; do
  for m in 1 0; do
    RINGDP_F32_CONV1_WPARTS=$m timeout -k 10 300 python -u bench.py --dtype fp32 --batch-per-rank 100 --steps 200 --warmup 20 --comm-stats-steps 0 > $O/b100_s$m.$r.json 2>>$O/b.err || exit 1
    tail -1 $O/b100_s$m.$r.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('B=100 slices=$m', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 python -u bench.py --dtype fp32 --comm-stats-steps 0 > $O/b65536.json 2>>$O/b.err || exit 1
tail -1 $O/b65536.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('B=65536', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --dtype fp32 --batch-per-rank 100 --steps 200 --warmup 20 --comm-stats-steps 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); python tools/prof_summary.py $f 40 > $O/k_100.md; head -22 $O/k_100.md
