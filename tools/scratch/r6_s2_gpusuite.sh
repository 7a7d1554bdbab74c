#!/bin/bash
# round 6 (session 2): the whole GPU suite on the final tree
set -o pipefail
O=gpurun_out/r6_s2_gpusuite
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
