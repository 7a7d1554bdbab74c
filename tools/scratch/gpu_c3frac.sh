#!/bin/bash
# conv3/conv2 backward role-split sweep (kbench medians): bash tools/gpu_c3frac.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in ${FRACS:-0.5 0.55 0.5 0.55}; do
  echo -n "c3=$f c2=${C2F:-0.55} "
  RINGDP_C3_DGRAD_FRAC=$f RINGDP_C2_DGRAD_FRAC=${C2F:-0.55} timeout -k 10 120 python tools/kbench.py 32768 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: v['us'] for k, v in d.items() if isinstance(v, dict) and k.startswith(('conv3_fc_bwd', 'conv2_bwd'))}, d['total_us'])" || exit 1
done
