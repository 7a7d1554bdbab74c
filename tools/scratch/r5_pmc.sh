#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) for ConvNet ops: r5_pmc.sh NAME B op...
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
N=$1; B=$2; shift 2
O=$R/gpurun_out/$N; mkdir -p $O
for OP in "$@"; do
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc_${OP}_$i -o run -- python3 $R/tools/pmc_run.py $OP $B 3 > $O/${OP}_$i.log 2>&1 || { echo "group $i failed"; tail -5 $O/${OP}_$i.log; exit 1; }
  f=$(find /tmp/pmc_${OP}_$i -name "*counter_collection.csv" | head -1)
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
done
grep -h "bwd8\|conv3_bwd\|conv12" $O/*.txt | cut -c1-400
