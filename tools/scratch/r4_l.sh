#!/bin/bash
# fused forward v2 schedule (consumer epilogue beside conv1, k-steps beside pool2), headline A/B
set -o pipefail
O=gpurun_out/r4l; mkdir -p $O; rm -f $O/times.jsonl
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_convnet_kernels_gpu.py -k "fused_forward" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
for B in 65536 1024 100; do
  timeout -k 10 120 python tools/op_time.py fwd_sep $B 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
  timeout -k 10 120 python tools/op_time.py fwd_fused $B 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
done
RINGDP_FF_INPACK=0 timeout -k 10 120 python tools/op_time.py fwd_fused 100 20 | sed 's/}/, "inpack": 0}/' >> $O/times.jsonl 2>>$O/t.err || exit 1
for a in 1 2; do
  RINGDP_FF_ABLATE=$a timeout -k 10 120 python tools/op_time.py fwd_fused 65536 20 | sed "s/}/, \"ablate\": $a}/" >> $O/times.jsonl 2>>$O/t.err || exit 1
done
cat $O/times.jsonl
for f in 0 1; do
  RINGDP_CN_FUSED_FWD=$f timeout -k 10 200 python bench.py --steps 20 > $O/b_$f.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "fused=$f $(tail -1 $O/b_$f.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"])')"
done
RINGDP_CN_FUSED_FWD=1 timeout -k 10 300 $T tests/test_convnet_model_gpu.py > $O/model.log 2>&1; tail -2 $O/model.log
timeout -k 10 300 $T tests/test_nn_kernels_gpu.py -k "trajectory" -s > $O/fp8traj.log 2>&1; tail -2 $O/fp8traj.log
timeout -k 10 300 python tools/comm_bench.py --gpus 2 --backend xgmi --dtypes fp32 --sizes 454720,77312,377408,26214400,77312 > $O/comm_xgmi_ws2.jsonl 2>$O/comm.err || { tail -5 $O/comm.err; exit 1; }
grep '"impl"' $O/comm_xgmi_ws2.jsonl
echo ALLDONE
