#!/bin/bash
# Round-2 evidence, second half (bench configs after the ConvNet ones) with periodic Python stack dumps
# (RINGDP_BENCH_STACKS_S) so a run that stops progressing names where; then the ConvNet step profiles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ev
mkdir -p $OUT
export TMPDIR=/tmp RINGDP_BENCH_STACKS_S=40
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v '^ ' $OUT/$name.log | tail -3 | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run bench_convnet_fp32 170 python bench.py --dtype fp32 --steps 20 --warmup 5
run bench_resnet18 170 python bench.py --model resnet18 --steps 30 --warmup 5
run bench_resnet50 200 python bench.py --model resnet50 --steps 10 --warmup 3
run bench_vit 200 python bench.py --model vit_b_16 --steps 10 --warmup 3
run bench_vit_fp8 200 python bench.py --model vit_b_16 --dtype fp8 --steps 10 --warmup 3
unset RINGDP_BENCH_STACKS_S
bash tools/gpu_prof_step.sh
echo ALLDONE
