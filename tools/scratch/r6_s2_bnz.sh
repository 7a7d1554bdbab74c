#!/bin/bash
# round 6 (session 2): BN + ReLU backward without a residual reads dy and z only (mask from z and the forward's
# scale / shift), no stored pre-activation gradient - NN / parity tests, ResNet-18 / -50 benches, ResNet-50 table
set -o pipefail
O=gpurun_out/r6_s2_bnz
R=$PWD
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_nn_kernels_gpu.py tests/test_model_parity_gpu.py > $O/tests_nn.txt 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 180 python bench.py --model resnet50 --steps 30 --comm-stats-steps 0 > $O/rn50_$r.json 2>> $O/b.err || exit 1
  timeout -k 10 120 python bench.py --model resnet18 --steps 200 --comm-stats-steps 0 > $O/rn18_$r.json 2>> $O/b.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $R && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_rn50 -o run -- python3 bench.py --model resnet50 --steps 20 --warmup 3 --comm-stats-steps 0 > $O/prof.log 2>&1 || exit 1
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
echo DONE >> $O/summary.txt
