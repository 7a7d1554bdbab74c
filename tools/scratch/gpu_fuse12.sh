#!/bin/bash
# Fused conv2-backward + conv1-wgrad: kernel numerics, model tests, then A/B of the ConvNet step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/f12
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v '^ ' $OUT/$name.log | tail -${TAILN:-1} | cut -c1-${CUT:-300}; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=4 run tests 400 python -u -m pytest tests/test_convnet_kernels_gpu.py tests/test_convnet_model_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
export CUT=220
run b_fused 150 python bench.py --steps 200 --warmup 20
RINGDP_CN_FUSE12=0 run b_sep 150 python bench.py --steps 200 --warmup 20
run b100_fused 150 python bench.py --steps 500 --warmup 20 --batch-per-rank 100
run b4096_fused 150 python bench.py --steps 300 --warmup 20 --batch-per-rank 4096
RINGDP_CN_FUSE12=0 run b4096_sep 150 python bench.py --steps 300 --warmup 20 --batch-per-rank 4096
for f in ${FRACS:-0.58 0.66 0.70}; do RINGDP_C12_DGRAD_FRAC=$f run b_frac$f 150 python bench.py --steps 200 --warmup 20; done
echo ALLDONE
