#!/bin/bash
# round 6 (session 2): fp32 pool slab forward templated on the slice count
set -o pipefail
O=gpurun_out/r6_s2_ps
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
R=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_convnet_fp32_gpu.py > $O/tests_f32.txt 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 120 python bench.py --batch-per-rank 100 --dtype fp32 --steps 2000 --comm-stats-steps 0 > $O/f32_b100_$r.json 2>> $O/b.err || exit 1
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_f32 -o run -- python3 bench.py --batch-per-rank 100 --dtype fp32 --steps 500 --comm-stats-steps 0 > $O/prof_f32.log 2>&1 || exit 1
for f in $O/*.json; do python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f',d['value'],d['ms_per_step'])"; done > $O/summary.txt
