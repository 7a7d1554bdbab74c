#!/bin/bash
set -o pipefail
O=gpurun_out/r6_s2_ffst
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
RINGDP_EXT_PATH=vtmp/ffst.so timeout -k 10 120 python tools/scratch/r6_s2_ffst.py > $O/stamps.txt 2>&1
