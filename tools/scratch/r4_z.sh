#!/bin/bash
# fp8 256 kernel: conflict-free chunk swizzle + grouped tile order, A/B by env
set -o pipefail
O=gpurun_out/r4z; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_nn_kernels_gpu.py -k "fp8" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
for cfg in "0 1" "1 1" "0 4" "1 4" "1 8"; do set -- $cfg
  RINGDP_FP8_SWZ=$1 RINGDP_FP8_GROUP_M=$2 timeout -k 10 200 python -u tools/gemm_bench.py --vit-fp8 > $O/gemm_$1_$2.log 2>&1 || exit 1
  echo "swz=$1 group=$2" >> $O/gemm.txt; cat $O/gemm_$1_$2.log >> $O/gemm.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES TCC_HIT_sum TCC_MISS_sum --output-format csv -d /tmp/pz -o run -- python3 $R/tools/pmc_gemm.py 8192 8192 8192 3 fp8 > $R/$O/pmc.log 2>&1 || exit 1
f=$(find /tmp/pz -name "*counter_collection.csv" | head -1); cp $f $R/$O/pmc_8192.csv
cd $R
for r in 1 2; do for v in "0 1" "1 4"; do set -- $v
  RINGDP_FP8_SWZ=$1 RINGDP_FP8_GROUP_M=$2 timeout -k 10 300 python -u bench.py --model vit_b_16 --dtype fp8 --steps 10 2>>$O/b.err | grep metric | sed "s/^/swz$1_g$2 /" >> $O/ab.txt || exit 1
done; done
echo ALLDONE
cat $O/gemm.txt; cut -c1-140 $O/ab.txt
