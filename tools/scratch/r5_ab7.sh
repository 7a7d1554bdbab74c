#!/bin/bash
# GEMM tails (parallel column tail <= 32 rows), two-barrier fused BN backward: tests, ResNet-18 A/B, kernel table
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_ab7; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "nn_kernels or resnet or model_parity or forced_comm" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
B="timeout -k 10 300 python -u bench.py --model resnet18 --steps 50 --warmup 20"
for r in 1 2; do
  RINGDP_GEMM_TAILS=0 $B --comm-stream same > $O/r18_off$r.json 2>>$O/b.err || exit 1
  RINGDP_BN_BWD_FUSED=0 $B --comm-stream same > $O/r18_nobn$r.json 2>>$O/b.err || exit 1
  $B --comm-stream same > $O/r18_on$r.json 2>>$O/b.err || exit 1
  $B --comm-stream split > $O/r18_split$r.json 2>>$O/b.err || exit 1
  for f in off nobn on split; do python -c "import json;d=json.load(open('$O/r18_$f$r.json'));print('$f', d['value'], d['ms_per_step'])"; done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --model resnet18 --steps 20 --warmup 5 --comm-stream same > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); python tools/prof_summary.py $f 60 > $O/prof_r18.md; cat $O/prof_r18.md
