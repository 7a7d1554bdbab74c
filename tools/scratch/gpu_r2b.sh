#!/bin/bash
# New round-2 GPU tests first (watchdog, multi-rank harness at ws=1, coalescing, split), then the rest.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2b
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -4 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
run new_tests 600 python -u -m pytest tests/test_watchdog_gpu.py tests/test_multigpu_gpu.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider
run all_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider
echo ALLDONE
