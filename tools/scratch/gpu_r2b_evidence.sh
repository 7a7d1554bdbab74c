#!/bin/bash
# Round-2 evidence (third session): full GPU tests, smoke, every bench config, ConvNet step profiles.
# Stops at the first failure; each step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ev3
mkdir -p $OUT
export TMPDIR=/tmp RINGDP_BENCH_STACKS_S=60
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v '^ ' $OUT/$name.log | tail -1 | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
run smoke 300 python __graft_entry__.py smoke
run bench_convnet 300 python bench.py
run bench_convnet_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_convnet_b100 300 python bench.py --batch-per-rank 100 --steps 500 --warmup 20
run bench_convnet_fp32 300 python bench.py --dtype fp32 --steps 20 --warmup 5
run bench_resnet18 300 python bench.py --model resnet18 --steps 50 --warmup 5
run bench_resnet50 300 python bench.py --model resnet50 --steps 10 --warmup 3
run bench_vit 300 python bench.py --model vit_b_16 --steps 10 --warmup 3
run bench_vit_fp8 300 python bench.py --model vit_b_16 --dtype fp8 --steps 10 --warmup 3
unset RINGDP_BENCH_STACKS_S
bash tools/gpu_prof_step.sh
echo ALLDONE
