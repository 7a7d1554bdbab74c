#!/bin/bash
# round 6 (session 2): fused forward A/B - software-pipelined A-fragment reads in the conv3 (KPIPE) / conv2 (PPIPE)
# k-step loops (vtmp/*.so built by tools/build_variant.py with the macros)
set -o pipefail
O=gpurun_out/r6_s2_pipe
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
B="timeout -k 10 120 python bench.py --steps 200 --warmup 20 --comm-stats-steps 0"
for r in 1 2; do
  $B > $O/base_$r.json 2>> $O/b.err || exit 1
  for v in kpipe ppipe kppipe; do
    RINGDP_EXT_PATH=vtmp/$v.so $B > $O/${v}_$r.json 2>> $O/b.err || exit 1
  done
done
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
# fp32 whole-network node with the group-parallel multi-segment reduction
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_convnet_fp32_gpu.py > $O/tests_f32.txt 2>&1 && \
timeout -k 10 120 python bench.py --batch-per-rank 100 --dtype fp32 --steps 2000 --comm-stats-steps 0 > $O/f32_b100.json 2>> $O/b.err && \
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_f32 -o run -- python3 bench.py --batch-per-rank 100 --dtype fp32 --steps 500 --comm-stats-steps 0 > $O/prof_f32.log 2>&1
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
