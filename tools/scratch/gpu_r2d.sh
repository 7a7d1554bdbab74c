#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2d
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -4 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
run fp32_tests 400 python -u -m pytest tests/test_convnet_fp32_gpu.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider
run bench_fp32 300 python bench.py --dtype fp32 --steps 20 --warmup 5
run bench_fp32_b100 300 python bench.py --dtype fp32 --batch-per-rank 100 --steps 100 --warmup 10
echo ALLDONE
