#!/bin/bash
# ConvNet kernel/model tests + headline and reference-batch bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/q4
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v '^ ' $OUT/$name.log | tail -${TAILN:-1} | cut -c1-${CUT:-230}; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=3 run tests 400 python -u -m pytest tests/test_convnet_kernels_gpu.py tests/test_convnet_model_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
run bench 150 python bench.py --steps 200 --warmup 20
run bench2 150 python bench.py --steps 200 --warmup 20
run b100 150 python bench.py --steps 500 --warmup 20 --batch-per-rank 100
echo ALLDONE
