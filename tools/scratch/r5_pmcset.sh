#!/bin/bash
# several PMC sets in one call
set -o pipefail
R=${GRAFT_REPO_ROOT:-.}
bash $R/tools/scratch/r5_pmc2.sh r5_pmc_c3w 65536 conv3_fc_ce_bwd RINGDP_C3_ABLATE=3 && \
bash $R/tools/scratch/r5_pmc2.sh r5_pmc_c3 65536 conv3_fc_ce_bwd && \
bash $R/tools/scratch/r5_pmc2.sh r5_pmc_c12w 65536 conv12_bwd RINGDP_C12_ABLATE=3 && \
bash $R/tools/scratch/r5_pmc2.sh r5_pmc_c12 65536 conv12_bwd && \
bash $R/tools/scratch/r5_pmc2.sh r5_pmc_ff 65536 fwd_fused
