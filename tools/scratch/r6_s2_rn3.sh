#!/bin/bash
# round 6 (session 2): head backward with staged logits gradients; ConvNet tests at the pool2 split 800; ResNet-18
# bench + kernel table
set -o pipefail
O=gpurun_out/r6_s2_rn3
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_nn_kernels_gpu.py -k "classifier_head or resnet" > $O/tests_head.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_convnet_model_gpu.py tests/test_convnet_kernels_gpu.py tests/test_model_parity_gpu.py > $O/tests_cn.txt 2>&1 && \
for r in 1 2; do
  timeout -k 10 120 python bench.py --model resnet18 --steps 200 --comm-stats-steps 0 > $O/rn18_$r.json 2>> $O/b.err || exit 1
done && \
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rn18 -o run -- python3 bench.py --model resnet18 --steps 100 --comm-stats-steps 0 > $O/prof_rn18.log 2>&1
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
