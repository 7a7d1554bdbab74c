#!/bin/bash
# PMC counter passes for one ConvNet op (tools/pmc_run.py), one rocprofv3 run per counter group:
#   bash tools/pmc_op.sh <op> [B] [tag]
# Writes gpurun_out/pmc/<tag>/<op>.txt: one line per kernel, counters averaged over the calls
# (whole-chip sums; SQ_* cycle counters are quad-cycles except SQ_VALU_MFMA_BUSY_CYCLES).
# Group limits per pass (rocprofv3 does not split): <= 8 SQ_, <= 4 TCC_ (FETCH_SIZE = 3, WRITE_SIZE = 2).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
OP=$1; B=${2:-65536}; TAG=${3:-cur}
OUT=$R/gpurun_out/pmc/$TAG
mkdir -p $OUT
: > $OUT/$OP.txt
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc_${OP}_$i -o run -- python3 $R/tools/pmc_run.py $OP $B 3 > $OUT/${OP}_$i.log 2>&1 || { echo "group $i failed"; tail -5 $OUT/${OP}_$i.log; exit 1; }
  f=$(find /tmp/pmc_${OP}_$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY' >> $OUT/$OP.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"][:70]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k, d in agg.items():
    n = max(1, len(disp[k]))
    print(k, {c: round(v / n, 1) for c, v in d.items()})
PY
done
cat $OUT/$OP.txt
