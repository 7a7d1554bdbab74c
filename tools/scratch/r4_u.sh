#!/bin/bash
set -o pipefail
O=gpurun_out/r4u; mkdir -p $O; rm -f $O/times.jsonl
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_convnet_kernels_gpu.py tests/test_convnet_model_gpu.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  timeout -k 10 120 python tools/op_time.py conv3_fc_ce_bwd 65536 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
done
cat $O/times.jsonl
timeout -k 10 200 python bench.py > $O/b.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
echo "bench $(tail -1 $O/b.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"])')"
timeout -k 10 200 python bench.py --batch-per-rank 100 --steps 300 > $O/b100.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
echo "B=100 $(tail -1 $O/b100.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"])')"
timeout -k 10 300 bash tools/pmc_op.sh conv3_fc_ce_bwd 65536 r4u > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
grep conv3_bwd gpurun_out/pmc/r4u/conv3_fc_ce_bwd.txt | head -2
echo ALLDONE
