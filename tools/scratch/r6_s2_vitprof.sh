#!/bin/bash
# round 6 (session 2): ViT-B/16 kernel tables (bf16, fp8)
set -o pipefail
O=gpurun_out/r6_s2_vitprof
R=$PWD
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd $R && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_vit -o run -- python3 bench.py --model vit_b_16 --steps 20 --warmup 3 --comm-stats-steps 0 > $O/prof_vit.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_vit8 -o run -- python3 bench.py --model vit_b_16 --dtype fp8 --steps 20 --warmup 3 --comm-stats-steps 0 > $O/prof_vit8.log 2>&1
echo DONE > $O/done.txt
