#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2c
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -4 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
run p2p_tests 300 python -u -m pytest tests/test_p2p_allreduce_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
run comm_bench 200 python tools/comm_bench.py --iters 10
echo ALLDONE
