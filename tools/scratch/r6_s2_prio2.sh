#!/bin/bash
# round 6 (session 2): wave issue priority A/B through the run-time ablate bits (results unchanged):
# RINGDP_FF_ABLATE 16 / 32 / 48 (fused forward consumer phase 3 / producer phases 1-2 / both),
# RINGDP_C3_ABLATE=8 + RINGDP_C12_ABLATE=8 (backward dgrad roles' younger half); tests of the compile-time pool2
# split and the head backward first
set -o pipefail
O=gpurun_out/r6_s2_prio2
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_nn_kernels_gpu.py -k "classifier_head or resnet" > $O/tests_head.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_convnet_model_gpu.py tests/test_convnet_kernels_gpu.py > $O/tests_cn.txt 2>&1 || exit 1
B="timeout -k 10 120 python bench.py --steps 200 --warmup 20 --comm-stats-steps 0"
for r in 1 2; do
  $B > $O/base_$r.json 2>> $O/b.err || exit 1
  RINGDP_FF_ABLATE=16 $B > $O/ff16_$r.json 2>> $O/b.err || exit 1
  RINGDP_FF_ABLATE=32 $B > $O/ff32_$r.json 2>> $O/b.err || exit 1
  RINGDP_FF_ABLATE=48 $B > $O/ff48_$r.json 2>> $O/b.err || exit 1
  RINGDP_C3_ABLATE=8 RINGDP_C12_ABLATE=8 $B > $O/bwd8_$r.json 2>> $O/b.err || exit 1
done
timeout -k 10 120 python bench.py --model resnet18 --steps 200 --comm-stats-steps 0 > $O/rn18.json 2>> $O/b.err && \
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rn18 -o run -- python3 bench.py --model resnet18 --steps 100 --comm-stats-steps 0 > $O/prof_rn18.log 2>&1
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
