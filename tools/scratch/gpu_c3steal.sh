#!/bin/bash
# conv3 backward: share of data-gradient images moved to the wgrad workgroups (kbench medians)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for f in ${STEALS:-0 0.1 0.15 0.2 0.25 0.3}; do
  echo -n "steal=$f "
  RINGDP_C3_STEAL=$f timeout -k 10 120 python tools/kbench.py 32768 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: v['us'] for k, v in d.items() if isinstance(v, dict) and k.startswith(('conv3_fc_bwd', 'conv2_bwd'))}, d['total_us'])" || exit 1
done
