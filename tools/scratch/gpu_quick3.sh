#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/q
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} $OUT/$name.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc; }
run tests 300 python -u -m pytest tests/test_convnet_kernels_gpu.py tests/test_convnet_model_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
run kbench 200 python tools/kbench.py 32768 100
run bench 200 python bench.py --steps 100 --warmup 10
run bench100 200 python bench.py --steps 300 --warmup 20 --batch-per-rank 100
echo ALLDONE
