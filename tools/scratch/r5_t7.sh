#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "convnet" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
bash tools/scratch/r5_ops.sh $1 "conv3_fc_ce_bwd X=0" "conv3_fc_ce_bwd RINGDP_C3_ABLATE=3" "conv3_fc_ce_bwd RINGDP_C3_ABLATE=4" "conv3_fc_ce_bwd RINGDP_C3_ABLATE=6" "conv12_bwd X=0" "conv12_bwd RINGDP_C12_ABLATE=3" "conv12_bwd RINGDP_C12_ABLATE=4" "conv12_bwd RINGDP_C12_ABLATE=7" "fwd_fused RINGDP_FF_P2=480" "fwd_fused RINGDP_FF_P2=560" "fwd_fused RINGDP_FF_P2=640" || exit 1
timeout -k 10 300 python -u bench.py > $O/b.json 2>>$O/b.err || exit 1
grep -h metric $O/b.json | cut -c100-200
