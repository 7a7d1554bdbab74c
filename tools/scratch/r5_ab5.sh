#!/bin/bash
# GEMM tails (split-K last arriver, BN prepare in the conv tail, one-launch BN backward), pipelined fc1,
# split-graph comm placement: GPU tests, fwd_fused A/B, ResNet-18 tails on/off, comm placement, kernel table
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_ab5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "nn_kernels or convnet_kernels or resnet or model_parity or forced_comm" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
for r in 1 2; do
  RINGDP_EXT_PATH=abv/base.so timeout -k 10 120 python tools/op_time.py fwd_fused 65536 40 | tee -a $O/ops.jsonl || exit 1
  timeout -k 10 120 python tools/op_time.py fwd_fused 65536 40 | tee -a $O/ops.jsonl || exit 1
done
for r in 1 2; do
  RINGDP_GEMM_TAILS=0 timeout -k 10 300 python -u bench.py --model resnet18 --steps 50 --warmup 20 --comm-stream same > $O/r18_base$r.json 2>>$O/b.err || exit 1
  timeout -k 10 300 python -u bench.py --model resnet18 --steps 50 --warmup 20 --comm-stream same > $O/r18_new$r.json 2>>$O/b.err || exit 1
  timeout -k 10 300 python -u bench.py --model resnet18 --steps 50 --warmup 20 > $O/r18_split$r.json 2>>$O/b.err || exit 1
  timeout -k 10 300 python -u bench.py --model resnet18 --steps 50 --warmup 20 --comm-stream side > $O/r18_side$r.json 2>>$O/b.err || exit 1
  cut -c1-150 $O/r18_base$r.json $O/r18_new$r.json $O/r18_split$r.json $O/r18_side$r.json
done
RINGDP_EXT_PATH=abv/base.so timeout -k 10 300 python -u bench.py --comm-stream same > $O/b_base.json 2>>$O/b.err || exit 1
timeout -k 10 300 python -u bench.py --comm-stream same > $O/b_new.json 2>>$O/b.err || exit 1
timeout -k 10 300 python -u bench.py > $O/b_split.json 2>>$O/b.err || exit 1
cut -c1-150 $O/b_base.json $O/b_new.json $O/b_split.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --model resnet18 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); python tools/prof_summary.py $f 40 > $O/prof_r18.md; cat $O/prof_r18.md
