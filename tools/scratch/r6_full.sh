#!/bin/bash
# round 6: full GPU suite (one process, per-test timeout), smoke, then the benches of every model
set -o pipefail
O=gpurun_out/r6_full
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 120 python bench.py > $O/b_convnet.json 2> $O/b_convnet.err && \
timeout -k 10 300 python bench.py --dtype fp32 --steps 30 --warmup 5 --comm-stats-steps 0 > $O/b_fp32.json 2> $O/b_fp32.err && \
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fp32 -o run -- python3 bench.py --dtype fp32 --steps 20 --warmup 5 --comm-stats-steps 0 > $O/prof.log 2>&1
