#!/bin/bash
# A/B of an extension variant against abv/base.so: ConvNet kernel tests, op timings, the headline bench.
# usage: r5_ab.sh NAME "ops..." [test-filter]
set -o pipefail
export TMPDIR=/tmp
N=$1; OPS=${2:-conv3_fc_ce_bwd}; TF=${3:-convnet}
O=gpurun_out/$N; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$TF" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
for r in 1 2; do for op in $OPS; do
  RINGDP_EXT_PATH=abv/base.so timeout -k 10 120 python tools/op_time.py $op 65536 40 | tee -a $O/ops.jsonl || exit 1
  timeout -k 10 120 python tools/op_time.py $op 65536 40 | tee -a $O/ops.jsonl || exit 1
done; done
for r in 1 2; do
  RINGDP_EXT_PATH=abv/base.so timeout -k 10 300 python -u bench.py > $O/b_base$r.json 2>>$O/b.err || exit 1
  timeout -k 10 300 python -u bench.py > $O/b_new$r.json 2>>$O/b.err || exit 1
  cut -c1-120 $O/b_base$r.json $O/b_new$r.json
done
