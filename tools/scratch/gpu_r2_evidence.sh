#!/bin/bash
# Round-2 evidence pass: full GPU tests, smoke, every bench config.  Stops at the first crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ev
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -1 $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
run smoke 300 python __graft_entry__.py smoke
run bench_convnet 300 python bench.py
run bench_convnet_b100 300 python bench.py --batch-per-rank 100 --steps 300 --warmup 20
run bench_convnet_fp32 300 python bench.py --dtype fp32 --steps 20 --warmup 5
run bench_resnet18 300 python bench.py --model resnet18 --steps 30 --warmup 5
run bench_resnet50 400 python bench.py --model resnet50 --steps 10 --warmup 3
run bench_vit 400 python bench.py --model vit_b_16 --steps 10 --warmup 3
run bench_vit_fp8 400 python bench.py --model vit_b_16 --dtype fp8 --steps 10 --warmup 3
echo ALLDONE
