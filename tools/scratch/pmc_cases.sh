#!/bin/bash
# LDS-conflict / L2 PMC pass over the bf16 GEMM and conv kernels (tools/pmc_cases.py)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcc; mkdir -p $O
for c in vit_fc1 vit_wgrad r50_c3 r50_pw r50_dgrad r50_wgrad; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum --output-format csv -d /tmp/pc_$c -o run -- python3 $R/tools/pmc_cases.py $c 3 > $O/$c.log 2>&1 || { echo "case $c failed"; tail -5 $O/$c.log; exit 1; }
  f=$(find /tmp/pc_$c -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$c" <<'PY' >> $O/cases.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:70]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    if any(s in k for s in ("gemm", "conv", "splitk")):
        print(sys.argv[2], k, {c: round(v / max(1, cnt[(k, c)])) for c, v in d.items()})
PY
done
cat $O/cases.txt
