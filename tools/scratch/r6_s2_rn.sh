#!/bin/bash
# round 6 (session 2): one-launch classifier head + folded BN statistics (ResNet-18): numerics, A/B bench,
# kernel table; then the fused-forward pool2 item split re-sweep (RINGDP_FF_P2)
set -o pipefail
O=gpurun_out/r6_s2_rn
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_nn_kernels_gpu.py -k "classifier_head or batchnorm or resnet or pools" tests/test_model_parity_gpu.py -k "resnet" > $O/tests.txt 2>&1 && \
timeout -k 10 120 python bench.py --model resnet18 --steps 100 --comm-stats-steps 0 > $O/b_rn18.json 2> $O/b_rn18.err && \
RINGDP_BN_FOLD=0 timeout -k 10 120 python bench.py --model resnet18 --steps 100 --comm-stats-steps 0 > $O/b_rn18_nofold.json 2> $O/b_rn18_nofold.err && \
timeout -k 10 120 python bench.py --model resnet18 --steps 100 --comm-stats-steps 0 > $O/b_rn18_2.json 2> $O/b_rn18_2.err && \
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rn18 -o run -- python3 bench.py --model resnet18 --steps 100 --comm-stats-steps 0 > $O/prof_rn18.log 2>&1 || exit 1
B="timeout -k 10 120 python bench.py --steps 100 --warmup 20 --comm-stats-steps 0"
for r in 1 2; do
  for v in 560 800 704; do
    RINGDP_FF_P2=$v $B > $O/p2_${v}_$r.json 2>> $O/b.err || exit 1
  done
done
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
