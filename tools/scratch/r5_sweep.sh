#!/bin/bash
# ConvNet kernel tests, then op timings of OP under each env setting: r5_sweep.sh NAME OP "ENV1" "ENV2" ...
set -o pipefail
export TMPDIR=/tmp
N=$1; OP=$2; shift 2
O=gpurun_out/$N; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "convnet" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
for r in 1 2; do for e in "$@"; do
  echo -n "$e : " | tee -a $O/ops.txt
  env $e timeout -k 10 120 python tools/op_time.py $OP 65536 40 | tee -a $O/ops.txt || exit 1
done; done
timeout -k 10 300 python -u bench.py > $O/b.json 2>>$O/b.err || exit 1
grep -h metric $O/b.json | cut -c100-200
