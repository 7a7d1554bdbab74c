#!/bin/bash
# A/B/C of extension builds on one box: abv/base.so, abv/new.so, in-tree.  r5_ab3.sh NAME "ops" [test-filter]
set -o pipefail
export TMPDIR=/tmp
N=$1; OPS=${2:-conv3_fc_ce_bwd}; TF=${3:-convnet}
O=gpurun_out/$N; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$TF" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
for r in 1 2; do for op in $OPS; do for v in abv/base.so abv/new.so ""; do
  echo -n "${v:-tree} " | tee -a $O/ops.txt
  RINGDP_EXT_PATH=$v timeout -k 10 120 python tools/op_time.py $op 65536 40 | tee -a $O/ops.txt || exit 1
done; done; done
for r in 1 2; do for v in abv/base.so abv/new.so ""; do
  RINGDP_EXT_PATH=$v timeout -k 10 300 python -u bench.py > $O/b.json 2>>$O/b.err || exit 1
  echo "${v:-tree} $(grep -o '"value": [0-9.]*' $O/b.json)" | tee -a $O/bench.txt
done; done
