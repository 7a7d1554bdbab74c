#!/bin/bash
set -o pipefail
O=gpurun_out/r4n; mkdir -p $O; rm -f $O/times.jsonl
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T -x tests/test_convnet_kernels_gpu.py -k "fused_forward" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
for p2 in 400 480 560 800; do
  RINGDP_FF_P2=$p2 timeout -k 10 120 python tools/op_time.py fwd_fused 65536 20 | sed "s/}/, \"p2\": $p2}/" >> $O/times.jsonl 2>>$O/t.err || exit 1
done
for a in 1 2; do
  RINGDP_FF_ABLATE=$a timeout -k 10 120 python tools/op_time.py fwd_fused 65536 20 | sed "s/}/, \"ablate\": $a}/" >> $O/times.jsonl 2>>$O/t.err || exit 1
done
timeout -k 10 120 python tools/op_time.py fwd_sep 65536 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
cat $O/times.jsonl
timeout -k 10 300 $T "tests/test_multigpu_gpu.py::test_ddp_equivalence_gpu" > $O/mgpu.log 2>&1; tail -3 $O/mgpu.log
timeout -k 10 1000 $T tests -m gpu > $O/gpu_tests.log 2>&1; tail -5 $O/gpu_tests.log
echo ALLDONE
