#!/bin/bash
# round 6 (session 2): fp32 reference batch - dedicated conv2 / conv3 forward kernels at B=100 (A/B only)
set -o pipefail
O=gpurun_out/r6_s2_f32s2
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
for r in 1 2; do
  timeout -k 10 120 python bench.py --batch-per-rank 100 --dtype fp32 --steps 2000 --comm-stats-steps 0 > $O/b100_def_$r.json 2>> $O/b.err && \
  RINGDP_F32_FWD_MIN_B=1 timeout -k 10 120 python bench.py --batch-per-rank 100 --dtype fp32 --steps 2000 --comm-stats-steps 0 > $O/b100_minb1_$r.json 2>> $O/b.err || exit 1
done && \
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
RINGDP_F32_FWD_MIN_B=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --batch-per-rank 100 --dtype fp32 --steps 500 --comm-stats-steps 0 > $O/prof.log 2>&1
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_nn_kernels_gpu.py -k "classifier_head" > $O/tests_head.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rn18 -o run -- python3 bench.py --model resnet18 --steps 100 --comm-stats-steps 0 > $O/prof_rn18.log 2>&1
