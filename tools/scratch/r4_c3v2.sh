#!/bin/bash
# conv3 backward v2: numerics tests, then same-box timing v1 vs v2, then the bench
set -o pipefail
O=gpurun_out/r4c3v2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_convnet_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv3" -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for v in 1 2; do
    RINGDP_C3_BWD=$v timeout -k 10 120 python tools/op_time.py conv3_fc_bwd 65536 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
    RINGDP_C3_BWD=$v timeout -k 10 120 python tools/op_time.py conv3_fc_bwd_w 65536 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
  done
done
cat $O/times.jsonl
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b_convnet.json 2>$O/b_convnet.err || exit 1; echo convnet $(grep -o '"value": [0-9.]*' $O/b_convnet.json)
echo ALLDONE
