#!/bin/bash
# One GPU round: tests, smoke, bench variants, rocprofv3 kernel stats.  Stops at the first crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 tmo=$2; shift 2
  echo "=== $name" | tee -a $OUT/summary.txt
  timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a $OUT/summary.txt
  tail -3 $OUT/$name.log | tee -a $OUT/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc" | tee -a $OUT/summary.txt; exit $rc; fi
  return 0
}
: > $OUT/summary.txt
for s in ${STEPS:-tests smoke bench}; do
  case $s in
    tests) step pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider ;;
    smoke) step smoke 300 python __graft_entry__.py smoke ;;
    bench) step bench_b100_eager 300 python bench.py --batch-per-rank 100 --steps 100 --warmup 10 --no-graph
           step bench_b1024_graph 300 python bench.py --batch-per-rank 1024 --steps 100 --warmup 10
           step bench_b100_graph 300 python bench.py --batch-per-rank 100 --steps 200 --warmup 10
           step bench_b4096_graph 300 python bench.py --batch-per-rank 4096 --steps 100 --warmup 10
           step bench_default 300 python bench.py ;;
    eager) step bench_b100_eager 300 python bench.py --batch-per-rank 100 --steps 100 --warmup 10 --no-graph
           step bench_b1024_eager 300 python bench.py --batch-per-rank 1024 --steps 100 --warmup 10 --no-graph
           step bench_b4096_eager 300 python bench.py --batch-per-rank 4096 --steps 50 --warmup 10 --no-graph
           step bench_b16384_eager 300 python bench.py --batch-per-rank 16384 --steps 20 --warmup 5 --no-graph ;;
    graphdiag) for lv in fwd loss bwd full; do step gdiag_$lv 300 env PYTHONPATH=. python tools/graph_diag.py $lv; done
           step gdiag_full_ddp 300 env PYTHONPATH=. python tools/graph_diag.py full ddp ;;
    kbench) step kbench 300 python tools/kbench.py ${KB:-100 1024 4096 16384} ;;
    prof)  step prof_b100 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_b100 -o run --output-format csv -- python bench.py --batch-per-rank 100 --steps 50 --warmup 5 --no-graph
           step prof_b4096 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_b4096 -o run --output-format csv -- python bench.py --batch-per-rank 4096 --steps 50 --warmup 5 --no-graph ;;
  esac
done
echo ALLDONE | tee -a $OUT/summary.txt
