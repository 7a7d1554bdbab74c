#!/bin/bash
# round 6 (session 2): one-launch conv weight pack with 16-B stores; fp32 tests with the group-parallel reduction
set -o pipefail
O=gpurun_out/r6_s2_pack2
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_nn_kernels_gpu.py -k "pack or resnet or classifier" > $O/tests_nn.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_model_parity_gpu.py tests/test_convnet_fp32_gpu.py > $O/tests_f32.txt 2>&1 && \
for r in 1 2; do
  timeout -k 10 120 python bench.py --model resnet18 --steps 200 --comm-stats-steps 0 > $O/rn18_one_$r.json 2>> $O/b.err && \
  RINGDP_PACK_SPLIT=1 timeout -k 10 120 python bench.py --model resnet18 --steps 200 --comm-stats-steps 0 > $O/rn18_split_$r.json 2>> $O/b.err || exit 1
done && \
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rn18 -o run -- python3 bench.py --model resnet18 --steps 100 --comm-stats-steps 0 > $O/prof_rn18.log 2>&1
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
