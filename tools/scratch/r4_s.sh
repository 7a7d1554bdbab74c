#!/bin/bash
set -o pipefail
O=gpurun_out/r4s; mkdir -p $O
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_convnet_kernels_gpu.py tests/test_convnet_model_gpu.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --batch-per-rank 100 --steps 300 > $O/b100.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
echo "B=100 $(tail -1 $O/b100.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"])')"
timeout -k 10 200 python bench.py > $O/b.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
echo "bench $(tail -1 $O/b.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"])')"
for op in fwd_fused conv3_fc_ce_bwd conv12_bwd; do
  timeout -k 10 300 bash tools/pmc_op.sh $op 65536 r4s > $O/pmc_$op.log 2>&1 || { tail -5 $O/pmc_$op.log; exit 1; }
done
ls gpurun_out/pmc/r4s
echo ALLDONE
