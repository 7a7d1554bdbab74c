#!/bin/bash
set -o pipefail
O=gpurun_out/r4j; mkdir -p $O; rm -f $O/times.jsonl
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_convnet_kernels_gpu.py -k "fused_forward" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
for B in 100 1024 65536; do
  timeout -k 10 120 python tools/op_time.py fwd_sep $B 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
  timeout -k 10 120 python tools/op_time.py fwd_fused $B 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
done
for a in 1 2; do
  RINGDP_FF_ABLATE=$a timeout -k 10 120 python tools/op_time.py fwd_fused 65536 20 | sed "s/}/, \"ablate\": $a}/" >> $O/times.jsonl 2>>$O/t.err || exit 1
done
for op in conv3_fc_bwd conv3_fc_ce_bwd; do
  timeout -k 10 120 python tools/op_time.py $op 65536 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
done
cat $O/times.jsonl
for f in 0 1; do
  RINGDP_CN_FUSED_FWD=$f timeout -k 10 200 python bench.py --batch-per-rank 100 --steps 300 > $O/b100_$f.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "fused=$f B=100 $(tail -1 $O/b100_$f.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"])')"
done
RINGDP_CN_FUSED_FWD=1 timeout -k 10 300 $T tests/test_convnet_model_gpu.py > $O/model.log 2>&1; tail -2 $O/model.log
# xgmi engine: exactness tests, then the all-reduce sweep at ws 2 (ranks share the GPU)
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_xgmi_gpu.py -k "exact" > $O/xgmi_tests.log 2>&1; rc=$?; tail -2 $O/xgmi_tests.log; [ $rc -eq 0 ] || exit 1
for nb in 64 256; do
  RINGDP_XGMI_BLOCKS=$nb timeout -k 10 300 python tools/comm_bench.py --gpus 2 --backend xgmi --dtypes fp32 > $O/comm_xgmi_ws2_b$nb.jsonl 2>$O/comm.err || { tail -5 $O/comm.err; exit 1; }
  echo "blocks $nb"; grep '"impl"' $O/comm_xgmi_ws2_b$nb.jsonl
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof32 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch-per-rank 100 --dtype fp32 --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof32.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof32.log; exit 1; }
echo ALLDONE
