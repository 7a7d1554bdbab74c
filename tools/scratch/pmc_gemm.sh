cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmcg_$i -o run -- python3 $R/tools/pmc_gemm.py 4096 4096 4096 3 > $R/gpurun_out/pmc/gemm_$i.log 2>&1 || { echo "group $i failed"; tail -5 $R/gpurun_out/pmc/gemm_$i.log; exit 1; }
  f=$(find /tmp/pmcg_$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY' >> $R/gpurun_out/pmc/gemm.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:120]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    if 'gemm' in k: print(k, {c: round(v / max(1, cnt[(k, c)]), 1) for c, v in d.items()})
PY
done
cat $R/gpurun_out/pmc/gemm.txt
