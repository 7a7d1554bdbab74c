#!/bin/bash
# xgmi defaults: the xgmi GPU tests (ranks share the GPU: the shared-device defaults), then the 128-block /
# 16 MiB configuration at ws2 / ws4 (explicit environment) on the all-reduce sweep
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_xgmi_def; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
for g in 2 4; do
  RINGDP_XGMI_BLOCKS=128 RINGDP_XGMI_SLOT_MB=16 timeout -k 10 200 python -u tools/comm_bench.py --gpus $g --backend xgmi --dtypes fp32,bf16 > $O/ws$g.jsonl 2>$O/ws$g.err || { tail -5 $O/ws$g.err; exit 1; }
  python -c "
import json
for l in open('$O/ws$g.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('ws$g', d.get('impl'), d.get('dtype'), d.get('bytes'), d.get('us_per_op'), d.get('algbw_GBps'))
"
done
