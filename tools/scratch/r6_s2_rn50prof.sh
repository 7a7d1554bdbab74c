#!/bin/bash
# round 6 (session 2): ResNet-50 kernel table
set -o pipefail
O=gpurun_out/r6_s2_rn50prof
R=$PWD
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd $R && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python3 bench.py --model resnet50 --steps 20 --warmup 3 --comm-stats-steps 0 > $O/prof.log 2>&1
echo DONE > $O/done.txt
