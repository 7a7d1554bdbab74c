#!/bin/bash
# N>1 captured-step comm placement: 2 ranks sharing the GPU on the xgmi backend (the RCCL path needs 2 GPUs)
set -o pipefail
O=gpurun_out/r4w; mkdir -p $O
for B in 65536 100; do
  RINGDP_GPU_BACKEND=xgmi timeout -k 10 400 python bench.py --gpus 2 --batch-per-rank $B --steps 20 > $O/b2_$B.json 2>$O/b2_$B.err || { tail -5 $O/b2_$B.err; exit 1; }
  tail -1 $O/b2_$B.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"], d["config"]["comm"])'
done
echo ALLDONE
