#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/q
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-3} $OUT/$name.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc; }
run tests 300 python -u -m pytest tests/test_convnet_kernels_gpu.py tests/test_convnet_model_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
for f in 0.4 0.5 0.6 0.7; do TAILN=1 run kbench_$f 200 env RINGDP_C3_DGRAD_FRAC=$f python tools/kbench.py 32768; done
TAILN=1 run bench 200 python bench.py --steps 50 --warmup 10
echo ALLDONE
