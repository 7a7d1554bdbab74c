#!/bin/bash
set -o pipefail
O=gpurun_out/r4c3v2d; mkdir -p $O; rm -f $O/times.jsonl
timeout -k 10 300 python -u -m pytest tests/test_convnet_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv3" -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
RINGDP_EXT_PATH=ab_so/stamp.so timeout -k 10 120 python tools/c3_stamps.py 65536 > $O/stamps.json 2>$O/stamps.err || { tail -3 $O/stamps.err; exit 1; }
cat $O/stamps.json
for r in 1 2; do
  RINGDP_C3_BWD=1 timeout -k 10 120 python tools/op_time.py conv3_fc_bwd 65536 15 >> $O/times.jsonl 2>>$O/t.err || exit 1
  RINGDP_C3_BWD=2 timeout -k 10 120 python tools/op_time.py conv3_fc_bwd 65536 15 >> $O/times.jsonl 2>>$O/t.err || exit 1
  RINGDP_C3_BWD=2 timeout -k 10 120 python tools/op_time.py conv3_fc_bwd_w 65536 15 >> $O/times.jsonl 2>>$O/t.err || exit 1
done
cat $O/times.jsonl

timeout -k 10 300 python -u -m pytest tests/test_model_parity_gpu.py -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1; tail -12 $O/parity.log
echo ALLDONE
