#!/bin/bash
# xgmi backend at ws2 (two ranks on one GPU): RINGDP_XGMI_BLOCKS x RINGDP_XGMI_SLOT_MB sweep of the all-reduce
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_xgmi; mkdir -p $O
for blk in 64 128 256; do
  for slot in 4 16 32; do
    echo "== blocks $blk slot ${slot}MB" | tee -a $O/sweep.txt
    RINGDP_XGMI_BLOCKS=$blk RINGDP_XGMI_SLOT_MB=$slot timeout -k 10 150 python -u tools/comm_bench.py --gpus 2 --backend xgmi \
      --sizes 454720,4194304,26214400 --dtypes fp32 --reps 10 --iters 10 > $O/b${blk}_s${slot}.jsonl 2>$O/b${blk}_s${slot}.err || { tail -5 $O/b${blk}_s${slot}.err; exit 1; }
    python -c "
import json
for l in open('$O/b${blk}_s${slot}.jsonl'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(d.get('impl'), d.get('bytes'), d.get('us_per_op'), d.get('algbw_GBps'))
" | tee -a $O/sweep.txt
  done
done
