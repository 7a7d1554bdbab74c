#!/bin/bash
set -o pipefail
O=gpurun_out/r4r; mkdir -p $O
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_convnet_kernels_gpu.py tests/test_convnet_model_gpu.py tests/test_convnet_fp32_gpu.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --batch-per-rank 100 --steps 300 > $O/b100.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
echo "B=100 $(tail -1 $O/b100.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"])')"
timeout -k 10 300 python bench.py --batch-per-rank 100 --dtype fp32 --steps 300 > $O/b100_fp32.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
echo "B=100 fp32 $(tail -1 $O/b100_fp32.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"])')"
timeout -k 10 200 python bench.py > $O/b.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
echo "bench $(tail -1 $O/b.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"])')"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof100 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch-per-rank 100 --steps 300 > $GRAFT_REPO_ROOT/$O/prof100.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof100.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof32 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch-per-rank 100 --dtype fp32 --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof32.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof32.log; exit 1; }
echo ALLDONE
