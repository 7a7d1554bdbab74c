#!/bin/bash
# ConvNet tests + op timings + bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "convnet" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
bash tools/scratch/r5_ops.sh $1 "conv3_fc_ce_bwd X=0" "conv3_fc_ce_bwd RINGDP_C3_ABLATE=3" "conv3_fc_ce_bwd RINGDP_C3_DGRAD_FRAC=0.6" "conv12_bwd X=0" "conv12_bwd RINGDP_C12_ABLATE=3" "conv12_bwd RINGDP_C12_DGRAD_FRAC=0.65" "fwd_fused X=0" "fwd_fused RINGDP_CN_FC_FUSED_MAX=1000000" || exit 1
timeout -k 10 300 python -u bench.py > $O/b.json 2>>$O/b.err || exit 1
grep -h metric $O/b.json | cut -c100-200
