#!/bin/bash
# kernel tables: fp32 ConvNet B=65536, ResNet-18, ResNet-50, ViT fp8 (stats csv only: trace dbs are too big to copy back)
set -o pipefail
O=gpurun_out/r4x; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_$n -o run -- python3 $R/bench.py "$@" > $R/$O/p_$n.log 2>&1 || { tail -5 $R/$O/p_$n.log; return 1; }
  cp $(find /tmp/p_$n -name "*kernel_stats.csv" | head -1) $R/$O/${n}_kernel_stats.csv
}
run fp32 --dtype fp32 --steps 5 --warmup 2 && run r18 --model resnet18 --steps 20 && run r50 --model resnet50 --steps 10 && run vit8 --model vit_b_16 --dtype fp8 --steps 10 && echo ALLDONE
