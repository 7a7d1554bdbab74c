#!/bin/bash
# round 6 (session 2): re-validate the restored tree - full GPU suite, smoke, headline + reference-batch benches,
# kernel tables of the reference batch (bf16 and fp32)
set -o pipefail
O=gpurun_out/r6_s2_full
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 120 python bench.py > $O/b_convnet.json 2> $O/b_convnet.err && \
timeout -k 10 300 python bench.py --dtype fp32 --steps 30 --warmup 5 --comm-stats-steps 0 > $O/b_fp32.json 2> $O/b_fp32.err && \
timeout -k 10 120 python bench.py --batch-per-rank 100 --steps 2000 --comm-stats-steps 0 > $O/b_b100.json 2> $O/b_b100.err && \
timeout -k 10 120 python bench.py --batch-per-rank 100 --dtype fp32 --steps 2000 --comm-stats-steps 0 > $O/b_b100f32.json 2> $O/b_b100f32.err && \
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b100 -o run -- python3 bench.py --batch-per-rank 100 --steps 500 --comm-stats-steps 0 > $O/prof_b100.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b100f32 -o run -- python3 bench.py --batch-per-rank 100 --dtype fp32 --steps 500 --comm-stats-steps 0 > $O/prof_b100f32.log 2>&1
