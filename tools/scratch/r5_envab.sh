#!/bin/bash
# A/B of two environment settings of the in-tree extension: ConvNet kernel tests, op timings, headline bench.
# usage: r5_envab.sh NAME "ENV_A" "ENV_B" "ops..." [test-filter]
set -o pipefail
export TMPDIR=/tmp
N=$1; EA=$2; EB=$3; OPS=${4:-conv3_fc_ce_bwd}; TF=${5:-convnet}
O=gpurun_out/$N; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$TF" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
for r in 1 2; do for op in $OPS; do
  env $EA timeout -k 10 120 python tools/op_time.py $op 65536 40 | sed "s/^/A /" | tee -a $O/ops.txt || exit 1
  env $EB timeout -k 10 120 python tools/op_time.py $op 65536 40 | sed "s/^/B /" | tee -a $O/ops.txt || exit 1
done; done
for r in 1 2; do
  env $EA timeout -k 10 300 python -u bench.py > $O/b_A$r.json 2>>$O/b.err || exit 1
  env $EB timeout -k 10 300 python -u bench.py > $O/b_B$r.json 2>>$O/b.err || exit 1
  grep -h metric $O/b_A$r.json $O/b_B$r.json | cut -c100-200
done
