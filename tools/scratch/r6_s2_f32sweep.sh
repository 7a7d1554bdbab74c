#!/bin/bash
# round 6 (session 2): fp32 B=100 split re-sweep on the round-6 step (whole-network node, one reduction launch):
# weight-gradient slice depth (RINGDP_F32_WGRAD_MIN_K), forward / data-gradient k slices
set -o pipefail
O=gpurun_out/r6_s2_f32sweep
mkdir -p $O
export PYTHONPATH=$PWD
B="timeout -k 10 120 python bench.py --batch-per-rank 100 --dtype fp32 --steps 2000 --warmup 200 --comm-stats-steps 0"
run() { local n=$1; shift; env "$@" $B > $O/$n.json 2>> $O/b.err || exit 1; }
O2=${O}_2; mkdir -p $O2; O=$O2
for r in 1 2; do
  run base_$r X=1
  run wk192_$r RINGDP_F32_WGRAD_MIN_K=192
  run wk256_$r RINGDP_F32_WGRAD_MIN_K=256
  run wk320_$r RINGDP_F32_WGRAD_MIN_K=320
  run wk384_$r RINGDP_F32_WGRAD_MIN_K=384
done
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
echo DONE >> $O/summary.txt
RINGDP_F32_WGRAD_MIN_K=256 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_convnet_fp32_gpu.py > $O/tests_wk256.txt 2>&1
echo "tests rc=$?" >> $O/summary.txt
