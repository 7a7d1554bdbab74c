#!/bin/bash
# round 6 (session 2): sanity after the BN knob refactor - NN kernels, parity, smoke
set -o pipefail
O=gpurun_out/r6_s2_sanity
rm -rf $O; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_nn_kernels_gpu.py tests/test_model_parity_gpu.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 120 python bench.py --model resnet18 --steps 200 --comm-stats-steps 0 > $O/rn18.json 2>> $O/b.err || exit 1
echo DONE >> $O/tests.txt
