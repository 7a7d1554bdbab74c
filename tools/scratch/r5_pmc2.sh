#!/bin/bash
# PMC passes for one ConvNet op under an env setting: r5_pmc2.sh NAME B OP [VAR=VAL ...]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
N=$1; B=$2; OP=$3; shift 3
for kv in "$@"; do export "$kv"; done
O=$R/gpurun_out/$N; mkdir -p $O
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc_${N}_$i -o run -- python3 $R/tools/pmc_run.py $OP $B 3 > $O/${OP}_$i.log 2>&1 || { echo "group $i failed"; tail -5 $O/${OP}_$i.log; exit 1; }
  f=$(find /tmp/pmc_${N}_$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY' >> $O/${OP}.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    print(k, {c: round(v / max(1, cnt[(k, c)]), 1) for c, v in d.items()})
PY
done
grep -h "bwd8\|fused_fwd" $O/${OP}.txt | cut -c1-500
