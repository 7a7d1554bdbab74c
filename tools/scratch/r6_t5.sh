#!/bin/bash
# round 6: backward role-split knobs re-swept on the current tree (one at a time around the defaults)
set -o pipefail
O=gpurun_out/r6_t5
mkdir -p $O
export PYTHONPATH=$PWD
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 300 --warmup 20 --comm-stats-steps 0 > $O/$n.json 2> $O/$n.err
}
run base && run c3f50 RINGDP_C3_DGRAD_FRAC=0.5 && run c3f60 RINGDP_C3_DGRAD_FRAC=0.6 && \
run st05 RINGDP_C3_STEAL=0.05 && run st15 RINGDP_C3_STEAL=0.15 && \
run c2f50 RINGDP_C2_DGRAD_FRAC=0.5 && run c2f60 RINGDP_C2_DGRAD_FRAC=0.6 && run base2
