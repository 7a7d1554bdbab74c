#!/bin/bash
# Fork-free overlap (split graph segments): tests, ws1 forced-comm placement A/B (ResNet-18, ViT-B/16),
# ws2 on one GPU over the xgmi backend with a per-rank kernel trace (bucket collectives vs backward kernels)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_split3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "nn_kernels or forced_comm or xgmi or multigpu" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
val() { tail -1 $1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$1', d['value'], d['ms_per_step'], d['config']['comm'][-120:])"; }
B="timeout -k 10 300 python -u bench.py --model resnet18 --steps 50 --warmup 20"
for r in 1 2; do
  for m in same split; do $B --comm-stream $m > $O/r18_$m$r.json 2>>$O/b.err || exit 1; val $O/r18_$m$r.json; done
  RINGDP_SPLIT_MIN_US=0 $B --comm-stream split > $O/r18_forced$r.json 2>>$O/b.err || exit 1; val $O/r18_forced$r.json
done
timeout -k 10 300 python -u bench.py > $O/convnet.json 2>>$O/b.err || exit 1; val $O/convnet.json
V="timeout -k 10 300 python -u bench.py --model vit_b_16 --steps 10 --warmup 5"
for m in same split; do $V --comm-stream $m > $O/vit_$m.json 2>>$O/b.err || exit 1; val $O/vit_$m.json; done
# ws2 on the one GPU (xgmi backend), each rank under its own kernel trace
export RINGDP_GPU_BACKEND=xgmi MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 WORLD_SIZE=2
for rk in 0 1; do
  RANK=$rk LOCAL_RANK=$rk timeout -k 10 400 rocprofv3 --kernel-trace -d $O/ws2_r$rk -o run --output-format csv -- \
    python3 bench.py --model resnet18 --gpus 2 --steps 20 --warmup 10 --comm-stats-steps 0 > $O/ws2_r$rk.log 2>&1 &
done
wait %1; rc1=$?; wait %2; rc2=$?
echo "ws2 rc $rc1 $rc2"; tail -1 $O/ws2_r0.log | cut -c1-400
[ $rc1 -eq 0 ] && [ $rc2 -eq 0 ] || exit 1
