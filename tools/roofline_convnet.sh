#!/bin/bash
# Per-kernel roofline inputs for the ConvNet step at the bench batch: kernel time (kernel trace),
# HBM bytes (TCC FETCH_SIZE / WRITE_SIZE, one pass each: together they exceed the 4 TCC counters)
# and LDS bank conflicts.  One rocprofv3 run per counter group, each under its own time limit.
#   bash tools/roofline_convnet.sh [B]   -> gpurun_out/roofline/<op>_<pass>.csv + summary.jsonl
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
B=${1:-32768}
OUT=$R/gpurun_out/roofline
mkdir -p $OUT
: > $OUT/summary.jsonl
for op in ${OPS:-conv1_fwd conv2_fwd conv3_fc_fwd conv3_fc_bwd conv12_bwd}; do
  for pass in time fetch write lds; do
    case $pass in
      time)  args="--kernel-trace" ;;
      fetch) args="--pmc FETCH_SIZE" ;;
      write) args="--pmc WRITE_SIZE" ;;
      lds)   args="--pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES" ;;
    esac
    d=/tmp/rl_${op}_$pass
    rm -rf $d
    timeout -s KILL 120 rocprofv3 $args --output-format csv -d $d -o run -- python3 $R/tools/pmc_run.py $op $B 3 \
      > $OUT/${op}_$pass.log 2>&1 || { echo "$op $pass failed"; tail -5 $OUT/${op}_$pass.log; exit 1; }
    f=$(find $d -name "*counter_collection.csv" -o -name "*kernel_trace.csv" | head -1)
    cp "$f" $OUT/${op}_$pass.csv
    python3 - "$f" "$op" "$pass" <<'PY' >> $OUT/summary.jsonl
import csv, sys, json, collections
f, op, pas = sys.argv[1:4]
rows = list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r["Kernel_Name"].split("(")[0][-70:]
    if pas == "time":
        agg[k]["ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    else:
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(json.dumps({"op": op, "pass": pas, "kernel": k,
                      **{c: sum(v) / len(v) for c, v in d.items()}, "n": len(next(iter(d.values())))}))
PY
  done
done
echo ROOFLINE_DONE
