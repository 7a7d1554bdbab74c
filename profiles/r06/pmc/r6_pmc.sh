#!/bin/bash
# round 6: PMC passes of the headline ConvNet kernels (B=65536) for the before/after table
set -o pipefail
rm -rf gpurun_out/pmc/r6
bash tools/pmc_op.sh fwd_fused 65536 r6 && bash tools/pmc_op.sh conv3_fc_bwd 65536 r6 && bash tools/pmc_op.sh conv12_bwd 65536 r6
