#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/vit
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} $OUT/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run r18_noforce 300 python bench.py --model resnet18 --steps 30 --warmup 5 --no-force-comm
run r18_ringdp 300 env RINGDP_GEMM_BACKEND=ringdp python bench.py --model resnet18 --steps 30 --warmup 5
run r18_default 300 python bench.py --model resnet18 --steps 30 --warmup 5
run vit_fp8 300 python bench.py --model vit_b_16 --dtype fp8 --steps 10 --warmup 3
echo ALLDONE
