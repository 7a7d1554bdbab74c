#!/bin/bash
# A/B of whole-extension variants in abv/*.so on the ConvNet bench (alternating, same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S=ringdp/_C.cpython-310-x86_64-linux-gnu.so
cp $S /tmp/orig_C.so
for r in 1 2; do for v in "$@"; do
  if [ -n "${AB_CMD:-}" ]; then cp abv/$v.so $S && echo -n "$v " && timeout -k 10 120 $AB_CMD 2>>gpurun_out/ab_err.log || exit 1; continue; fi
  cp abv/$v.so $S || exit 1
  echo -n "$v "
  mkdir -p gpurun_out; timeout -k 10 120 python bench.py --steps 300 --warmup 30 --comm-stats-steps 0 ${BENCH_ARGS:-} 2>gpurun_out/ab_err.log | python -c "import json,sys; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]); print(d['ms_per_step'])" || exit 1
done; done
cp /tmp/orig_C.so $S
