#!/bin/bash
# SGD writes the ConvNet's packed weights: GPU tests, B=100 and B=65536 benches, B=100 kernel table
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_pack; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "convnet or xgmi_ddp or sgd or optim" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
val() { tail -1 $1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$1', d['value'], d['ms_per_step'])"; }
for r in 1 2; do
  RINGDP_CN_PACK_IN_SGD=0 timeout -k 10 300 python -u bench.py --batch-per-rank 100 --steps 2000 --warmup 200 > $O/b100_base$r.json 2>>$O/b.err || exit 1; val $O/b100_base$r.json
  timeout -k 10 300 python -u bench.py --batch-per-rank 100 --steps 2000 --warmup 200 > $O/b100_new$r.json 2>>$O/b.err || exit 1; val $O/b100_new$r.json
done
timeout -k 10 300 python -u bench.py > $O/b_new.json 2>>$O/b.err || exit 1; val $O/b_new.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof100 -o run --output-format csv -- python3 bench.py --batch-per-rank 100 --steps 200 --warmup 20 > $O/prof100.log 2>&1 || { tail -5 $O/prof100.log; exit 1; }
f=$(find $O/prof100 -name '*kernel_stats.csv' | head -1); python tools/prof_summary.py $f 20 > $O/prof_b100.md; cat $O/prof_b100.md
