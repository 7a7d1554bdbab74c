#!/bin/bash
# Round-2 first GPU pass: GPU tests, smoke, headline bench (forced comm at N=1 vs none), ref batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2a
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -2 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
run smoke 300 python __graft_entry__.py smoke
run bench_default 300 python bench.py --steps 50 --warmup 10
run bench_noforce 300 python bench.py --steps 50 --warmup 10 --no-force-comm
run bench_b100 300 python bench.py --batch-per-rank 100 --steps 200 --warmup 20
echo ALLDONE
