#!/bin/bash
# GEMM tails with device-scope (SC1) hand-off instead of agent fences: tests, ResNet-18 tails off/on,
# comm placement split/same/side, R18 kernel table, B=100 ConvNet kernel table
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_ab6; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "nn_kernels or resnet or model_parity or forced_comm" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
for r in 1 2; do
  RINGDP_GEMM_TAILS=0 timeout -k 10 300 python -u bench.py --model resnet18 --steps 50 --warmup 20 --comm-stream same > $O/r18_base$r.json 2>>$O/b.err || exit 1
  timeout -k 10 300 python -u bench.py --model resnet18 --steps 50 --warmup 20 --comm-stream same > $O/r18_new$r.json 2>>$O/b.err || exit 1
  timeout -k 10 300 python -u bench.py --model resnet18 --steps 50 --warmup 20 --comm-stream split > $O/r18_split$r.json 2>>$O/b.err || exit 1
  timeout -k 10 300 python -u bench.py --model resnet18 --steps 50 --warmup 20 --comm-stream side > $O/r18_side$r.json 2>>$O/b.err || exit 1
  cut -c1-150 $O/r18_base$r.json $O/r18_new$r.json $O/r18_split$r.json $O/r18_side$r.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --model resnet18 --steps 20 --warmup 5 --comm-stream same > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); python tools/prof_summary.py $f 40 > $O/prof_r18.md; cat $O/prof_r18.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof100 -o run --output-format csv -- python3 bench.py --batch-per-rank 100 --steps 200 --warmup 20 --comm-stream same > $O/prof100.log 2>&1 || { tail -5 $O/prof100.log; exit 1; }
f=$(find $O/prof100 -name '*kernel_stats.csv' | head -1); python tools/prof_summary.py $f 20 > $O/prof_b100.md; cat $O/prof_b100.md
