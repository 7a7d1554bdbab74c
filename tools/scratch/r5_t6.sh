#!/bin/bash
# dgrad-only timings / PMC of the conv3 and conv12 backward (wgrad ablated)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-.}
bash $R/tools/scratch/r5_ops.sh r5_t6 "conv3_fc_ce_bwd RINGDP_C3_ABLATE=4" "conv3_fc_ce_bwd RINGDP_C3_ABLATE=5" "conv3_fc_ce_bwd RINGDP_C3_ABLATE=6" "conv12_bwd RINGDP_C12_ABLATE=4" "conv12_bwd RINGDP_C12_ABLATE=5" "conv12_bwd RINGDP_C12_ABLATE=6" "conv12_bwd RINGDP_C12_ABLATE=7" && \
bash $R/tools/scratch/r5_pmc2.sh r5_pmc_c12d 65536 conv12_bwd RINGDP_C12_ABLATE=4 && \
bash $R/tools/scratch/r5_pmc2.sh r5_pmc_c3d 65536 conv3_fc_ce_bwd RINGDP_C3_ABLATE=4
