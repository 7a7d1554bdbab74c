#!/bin/bash
# round 6 (session 2): conv3 steal share 0.07 - ConvNet GPU tests, smoke, headline bench, kernel table
set -o pipefail
O=gpurun_out/r6_s2_steal
R=$PWD
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_convnet_kernels_gpu.py tests/test_convnet_model_gpu.py tests/test_model_parity_gpu.py > $O/tests_cn.txt 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 120 python bench.py --comm-stats-steps 20 > $O/b_convnet_$r.json 2>> $O/b.err || exit 1
done
timeout -k 10 120 python bench.py --batch-per-rank 100 --steps 2000 --warmup 200 --comm-stats-steps 20 > $O/b_b100.json 2>> $O/b.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $R && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_convnet -o run -- python3 bench.py --steps 200 --comm-stats-steps 0 > $O/prof.log 2>&1 || exit 1
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
echo DONE >> $O/summary.txt
