#!/bin/bash
# fused forward: separate-pack mode, role ablations; fc_bwd with CE fused vs plain
set -o pipefail
O=gpurun_out/r4h; mkdir -p $O; rm -f $O/times.jsonl
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_convnet_kernels_gpu.py -k "fused_forward" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
for B in 65536 100; do
  timeout -k 10 120 python tools/op_time.py fwd_sep $B 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
  for a in 0 1 2 3; do
    RINGDP_FF_ABLATE=$a timeout -k 10 120 python tools/op_time.py fwd_fused $B 20 | sed "s/}/, \"ablate\": $a}/" >> $O/times.jsonl 2>>$O/t.err || exit 1
  done
  RINGDP_FF_INPACK=1 timeout -k 10 120 python tools/op_time.py fwd_fused $B 20 | sed "s/}/, \"inpack\": 1}/" >> $O/times.jsonl 2>>$O/t.err || exit 1
done
for op in conv3_fc_bwd conv3_fc_ce_bwd; do
  timeout -k 10 120 python tools/op_time.py $op 65536 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
done
cat $O/times.jsonl
echo ALLDONE
# xgmi engine: exactness tests, then the all-reduce sweep at ws 2 (ranks share the GPU), blocks 64 / 256
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_xgmi_gpu.py -k "exact" > $O/xgmi_tests.log 2>&1; rc=$?; tail -2 $O/xgmi_tests.log; [ $rc -eq 0 ] || exit 1
for nb in 64 256; do
  RINGDP_XGMI_BLOCKS=$nb timeout -k 10 300 python tools/comm_bench.py --gpus 2 --backend xgmi --dtypes fp32 > $O/comm_xgmi_ws2_b$nb.jsonl 2>$O/comm.err || { tail -5 $O/comm.err; exit 1; }
  echo "blocks $nb"; grep '"impl"' $O/comm_xgmi_ws2_b$nb.jsonl
done
echo ALLDONE2
