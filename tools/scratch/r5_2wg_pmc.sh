#!/bin/bash
# PMC passes: the 256x256 one-workgroup GEMM vs the 256x128 two-workgroup one (8192^3 and ViT fc1 forward)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/r5_2wg_pmc; mkdir -p $OUT
export RINGDP_BF16_TILE=256
for shape in "8192 8192 8192 3" "25216 3072 768 5"; do
  for m in 0 1; do
    export RINGDP_GEMM_2WG=$m
    tag="$(echo $shape | cut -d' ' -f1-3 | tr ' ' x)_2wg$m"
    i=0
    for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
               "TCC_HIT_sum TCC_MISS_sum SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE"; do
      i=$((i+1))
      timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d /tmp/p_${tag}_$i -o run -- python3 $R/tools/pmc_gemm.py $shape > $OUT/${tag}_$i.log 2>&1 || { echo "group $i failed"; tail -5 $OUT/${tag}_$i.log; exit 1; }
      f=$(find /tmp/p_${tag}_$i -name "*counter_collection.csv" | head -1)
      python3 - "$f" "$tag" <<'PY' >> $OUT/pmc.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    name = r["Kernel_Name"]
    if "gemm_bf16" not in name:
        continue
    k = name[name.index("gemm_bf16"):][:30]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r.get("Dispatch_Id", ""))
for k, d in agg.items():
    n = max(1, len(disp[k]))
    print(sys.argv[2], k, " ".join(f"{c}={v / n:.4g}" for c, v in sorted(d.items())))
PY
    done
  done
done
cat $OUT/pmc.txt
