#!/bin/bash
# fused forward: numerics vs the three-launch path, op timing, bench A/B at B=65536 and B=100
set -o pipefail
O=gpurun_out/r4g; mkdir -p $O; rm -f $O/times.jsonl
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_convnet_kernels_gpu.py -k "fused_forward" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
for B in 65536 100; do
  for op in fwd_sep fwd_fused; do
    timeout -k 10 120 python tools/op_time.py $op $B 20 >> $O/times.jsonl 2>>$O/t.err || exit 1
  done
done
cat $O/times.jsonl
for f in 0 1; do
  RINGDP_CN_FUSED_FWD=$f timeout -k 10 200 python bench.py --steps 20 > $O/b_$f.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "fused=$f $(python -c "import json;d=json.load(open('$O/b_$f.json'));print(d['value'], d['ms_per_step'])")"
  RINGDP_CN_FUSED_FWD=$f timeout -k 10 200 python bench.py --batch-per-rank 100 --steps 300 > $O/b100_$f.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "fused=$f B=100 $(python -c "import json;d=json.load(open('$O/b100_$f.json'));print(d['ms_per_step'])")"
done
RINGDP_CN_FUSED_FWD=1 timeout -k 10 300 $T tests/test_convnet_model_gpu.py > $O/model.log 2>&1; tail -3 $O/model.log
echo ALLDONE
