#!/bin/bash
# round 6 (session 2): ViT-B/16 256x256-kernel routing threshold re-sweep (bf16 and fp8)
set -o pipefail
O=gpurun_out/r6_s2_vitfill
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
V="timeout -k 10 180 python bench.py --model vit_b_16 --steps 30 --comm-stats-steps 0"
run() { local n=$1 e=$2; shift 2; env $e $V "$@" > $O/$n.json 2>> $O/b.err || exit 1; }
run bf_base X=1
run bf_f40 RINGDP_BF16_256_FILL=0.40
run bf_f70 RINGDP_BF16_256_FILL=0.70
run bf_f90 RINGDP_BF16_256_FILL=0.90
run f8_base X=1 --dtype fp8
run f8_f40 RINGDP_FP8_256_FILL=0.40 --dtype fp8
run f8_f70 RINGDP_FP8_256_FILL=0.70 --dtype fp8
run f8_f90 RINGDP_FP8_256_FILL=0.90 --dtype fp8
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
echo DONE >> $O/summary.txt
