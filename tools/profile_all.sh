#!/bin/bash
# Collect the round's evidence on one GPU box: full GPU test suite, benches for every model config,
# rocprofv3 kernel stats for each model, kernel microbenchmarks.  Stops at the first crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 tmo=$2; shift 2
  echo "=== $name" | tee -a $OUT/summary.txt
  timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a $OUT/summary.txt
  tail -2 $OUT/$name.log | cut -c1-400 | tee -a $OUT/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc" | tee -a $OUT/summary.txt; exit $rc; fi
}
: > $OUT/summary.txt
for s in ${STEPS:-tests bench prof micro}; do
  case $s in
    tests) run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench) run bench_convnet 300 python bench.py
           run bench_convnet_b100 300 python bench.py --batch-per-rank 100 --steps 300 --warmup 20
           run bench_resnet18 300 python bench.py --model resnet18 --steps 30 --warmup 5
           run bench_resnet50 400 python bench.py --model resnet50 --steps 10 --warmup 3
           run bench_vit 400 python bench.py --model vit_b_16 --steps 10 --warmup 3
           run bench_vit_fp8 400 python bench.py --model vit_b_16 --dtype fp8 --steps 10 --warmup 3 ;;
    prof)  run prof_convnet 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_convnet -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-graph
           run prof_resnet50 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_resnet50 -o run --output-format csv -- python3 bench.py --model resnet50 --steps 5 --warmup 2 --no-graph
           run prof_vit 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_vit -o run --output-format csv -- python3 bench.py --model vit_b_16 --steps 5 --warmup 2 --no-graph ;;
    micro) run kbench 300 python tools/kbench.py 100 1024 4096 16384
           run gemm_bench 300 python tools/gemm_bench.py ;;
  esac
done
echo ALLDONE | tee -a $OUT/summary.txt
