#!/bin/bash
# round 6 (session 2): fc1 forward with unconditional, issue-pinned prefetches (was: one register set in
# flight because a branch-guarded prefetch made the compiler wait vmcnt(0) before each group's last MFMA)
set -o pipefail
O=gpurun_out/r6_s2_fc1
R=$PWD
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_convnet_kernels_gpu.py tests/test_convnet_model_gpu.py > $O/tests_cn.txt 2>&1 || exit 1
B="timeout -k 10 120 python bench.py --steps 200 --warmup 20 --comm-stats-steps 0"
for r in 1 2; do $B > $O/b_$r.json 2>> $O/b.err || exit 1; done
cd /tmp && export TMPDIR=/tmp && cd $R && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python3 bench.py --steps 100 --comm-stats-steps 0 > $O/prof.log 2>&1
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
echo DONE >> $O/summary.txt
