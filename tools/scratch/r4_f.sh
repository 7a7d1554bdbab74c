#!/bin/bash
# parity tests (fp64 + bf16 oracle), B=100 slab-count sweep, fp32 B=100 bench
set -o pipefail
O=gpurun_out/r4f; mkdir -p $O
T="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T -s tests/test_model_parity_gpu.py > $O/parity.log 2>&1; echo "parity rc=$?"; grep -a "worst\|passed\|failed\|out " $O/parity.log
for w in "2 2" "4 2" "4 4" "8 4"; do
  set -- $w
  RINGDP_C3_WMIN=$1 RINGDP_C12_WMIN=$2 timeout -k 10 200 python bench.py --batch-per-rank 100 --steps 300 --warmup 20 > $O/b100_$1_$2.json 2>$O/b100.err || { tail -5 $O/b100.err; exit 1; }
  echo "wmin $1 $2: $(python -c "import json;d=json.load(open('$O/b100_$1_$2.json'));print(d['ms_per_step'])")"
done
timeout -k 10 300 python bench.py --batch-per-rank 100 --dtype fp32 --steps 300 --warmup 20 > $O/b100_fp32.json 2>$O/b100f.err || { tail -5 $O/b100f.err; exit 1; }
cat $O/b100_fp32.json
echo ALLDONE
