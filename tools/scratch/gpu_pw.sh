#!/bin/bash
# Pointwise convs on hipBLASLt: conv tests, per-shape timings per mode, ResNet-50/18 step A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pw
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 tmo=$2; shift 2; echo "=== $name"; timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v '^ ' $OUT/$name.log | tail -${TAILN:-1} | cut -c1-${CUT:-230}; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=3 run tests 300 python -u -m pytest tests/test_nn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "conv_fwd_dgrad or resnet"
for m in "" fd fdw; do RINGDP_PW_BLASLT=$m TAILN=9 CUT=400 run pw_$m 200 python tools/pw_bench.py 256; done
for m in "" fd fdw; do RINGDP_PW_BLASLT=$m run r50_$m 200 python bench.py --model resnet50 --steps 10 --warmup 3 --comm-stats-steps 0; done
for m in "" fd; do RINGDP_PW_BLASLT=$m run r18_$m 200 python bench.py --model resnet18 --steps 30 --warmup 5 --comm-stats-steps 0; done
echo ALLDONE
