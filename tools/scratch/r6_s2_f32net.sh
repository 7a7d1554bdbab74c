#!/bin/bash
# round 6 (session 2): fp32 whole-network cross-entropy node (one weight-gradient reduction launch per backward)
set -o pipefail
O=gpurun_out/r6_s2_f32net
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_convnet_fp32_gpu.py > $O/tests.txt 2>&1 && \
for r in 1 2; do
  timeout -k 10 120 python bench.py --batch-per-rank 100 --dtype fp32 --steps 2000 --comm-stats-steps 0 > $O/b100_net_$r.json 2>> $O/b.err && \
  RINGDP_F32_NET_NODE_MAX_B=0 timeout -k 10 120 python bench.py --batch-per-rank 100 --dtype fp32 --steps 2000 --comm-stats-steps 0 > $O/b100_layer_$r.json 2>> $O/b.err || exit 1
done && \
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --batch-per-rank 100 --dtype fp32 --steps 500 --comm-stats-steps 0 > $O/prof.log 2>&1
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
