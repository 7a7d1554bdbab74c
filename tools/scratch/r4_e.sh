#!/bin/bash
# round 4: fused head CE + deferred reduce (tests, B=100 bench + kernel trace), conv3 v2 timings, parity tests
set -o pipefail
O=gpurun_out/r4e; mkdir -p $O; rm -f $O/times.jsonl
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_convnet_model_gpu.py tests/test_convnet_kernels_gpu.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --batch-per-rank 100 --steps 300 --warmup 20 > $O/b100.json 2>$O/b100.err || { tail -5 $O/b100.err; exit 1; }
cat $O/b100.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof100 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch-per-rank 100 --steps 300 --warmup 20 > $GRAFT_REPO_ROOT/$O/prof100.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof100.log; exit 1; }
cd $GRAFT_REPO_ROOT
find $O/prof100 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/b100_kernel_stats.csv
RINGDP_EXT_PATH=ab_so/stamp.so timeout -k 10 120 python tools/c3_stamps.py 65536 > $O/stamps.json 2>$O/stamps.err || { tail -3 $O/stamps.err; exit 1; }
for r in 1 2; do
  RINGDP_C3_BWD=1 timeout -k 10 120 python tools/op_time.py conv3_fc_bwd 65536 15 >> $O/times.jsonl 2>>$O/t.err || exit 1
  RINGDP_C3_BWD=2 timeout -k 10 120 python tools/op_time.py conv3_fc_bwd 65536 15 >> $O/times.jsonl 2>>$O/t.err || exit 1
  RINGDP_C3_BWD=2 timeout -k 10 120 python tools/op_time.py conv3_fc_bwd_w 65536 15 >> $O/times.jsonl 2>>$O/t.err || exit 1
done
cat $O/times.jsonl
timeout -k 10 300 $T -s tests/test_model_parity_gpu.py > $O/parity.log 2>&1; tail -12 $O/parity.log
echo ALLDONE
