#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/vit
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} $OUT/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run tests 400 python -u -m pytest tests/test_nn_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
run vit_auto 300 python bench.py --model vit_b_16 --steps 10 --warmup 3
run vit_ringdp 300 env RINGDP_GEMM_BACKEND=ringdp python bench.py --model vit_b_16 --steps 10 --warmup 3
run r50 300 python bench.py --model resnet50 --steps 10 --warmup 3
run r18 300 python bench.py --model resnet18 --steps 30 --warmup 5
echo ALLDONE
