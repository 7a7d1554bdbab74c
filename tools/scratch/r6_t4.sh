#!/bin/bash
# round 6: A/B of fc1 inside the fused forward at B=65536 (after the cheaper pool2), with two pool2 splits
set -o pipefail
O=gpurun_out/r6_t4
mkdir -p $O
export PYTHONPATH=$PWD
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 300 --warmup 20 --comm-stats-steps 0 > $O/$n.json 2> $O/$n.err
}
run base && run fcin RINGDP_CN_FC_FUSED_MAX=1000000 && run fcin_p2_512 RINGDP_CN_FC_FUSED_MAX=1000000 RINGDP_FF_P2=512 && \
run fcin_p2_640 RINGDP_CN_FC_FUSED_MAX=1000000 RINGDP_FF_P2=640 && run base2 && run fcin2 RINGDP_CN_FC_FUSED_MAX=1000000
