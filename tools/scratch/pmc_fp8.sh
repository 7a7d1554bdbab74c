#!/bin/bash
# PMC passes over the fp8 256x256 GEMM: 8192^3 and the ViT fc2 forward shape
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc8
for shape in "8192 8192 8192" "25216 768 3072"; do
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TCC_EA0_RDREQ_sum TCC_REQ_sum"; do
  i=$((i+1))
  tag=$(echo $shape | tr ' ' x)_$i
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc8_$tag -o run -- python3 $R/tools/pmc_gemm.py $shape 3 fp8 > $R/gpurun_out/pmc8/$tag.log 2>&1 || { echo "group $tag failed"; tail -5 $R/gpurun_out/pmc8/$tag.log; exit 1; }
  f=$(find /tmp/pmc8_$tag -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$shape" <<'PY' >> $R/gpurun_out/pmc8/fp8.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    if 'gemm' in k: print(sys.argv[2], k, {c: round(v / max(1, cnt[(k, c)]), 1) for c, v in d.items()})
PY
done
done
cat $R/gpurun_out/pmc8/fp8.txt
