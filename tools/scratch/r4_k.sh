#!/bin/bash
# after force-inlining the role functions (conv2 wgrad role was a real call in conv12_bwd: flat LDS/global
# ops, callee-saved spills) and the xgmi kernels (XgArgs copied to scratch in every thread)
set -o pipefail
O=gpurun_out/r4k; mkdir -p $O; rm -f $O/times.jsonl
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_convnet_kernels_gpu.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
for op in conv12_bwd conv3_fc_ce_bwd fwd_sep; do
  timeout -k 10 120 python tools/op_time.py $op 65536 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
done
for B in 100 1024 65536; do
  timeout -k 10 120 python tools/op_time.py fwd_fused $B 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
done
timeout -k 10 120 python tools/op_time.py fwd_sep 100 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
cat $O/times.jsonl
timeout -k 10 200 python bench.py --steps 20 > $O/b.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
echo "bench $(tail -1 $O/b.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"])')"
for f in 0 1; do
  RINGDP_CN_FUSED_FWD=$f timeout -k 10 200 python bench.py --batch-per-rank 100 --steps 300 > $O/b100_$f.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "fused=$f B=100 $(tail -1 $O/b100_$f.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"])')"
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_xgmi_gpu.py > $O/xgmi_tests.log 2>&1; rc=$?; tail -2 $O/xgmi_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/comm_bench.py --gpus 2 --backend xgmi --dtypes fp32 > $O/comm_xgmi_ws2.jsonl 2>$O/comm.err || { tail -5 $O/comm.err; exit 1; }
grep '"impl"' $O/comm_xgmi_ws2.jsonl
timeout -k 10 300 $T tests/test_nn_kernels_gpu.py -k "trajectory" -s > $O/fp8traj.log 2>&1; tail -3 $O/fp8traj.log
echo ALLDONE
