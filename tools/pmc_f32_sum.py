"""Summarise rocprofv3 --pmc CSVs: per kernel name+grid, counters summed over the chip, averaged over calls."""
import collections
import csv
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "kern::" not in n:
            continue
        m = re.search(r"gemm_f32_kernel<(\d), (\d), [^,]*::(\w+)", n)
        k = (f"gemm{m.group(1)}{m.group(2)} {m.group(3)}" if m else n.split("(")[0].split("::")[-1]) + f" grid={r.get('Grid_Size', '')}"
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k, d in agg.items():
    v = {c: x / max(1, len(disp[(k, c)])) for c, x in d.items()}
    print(k)
    print("   ", {c: f"{x:.4g}" for c, x in sorted(v.items())})
    if v.get("SQ_INSTS_MFMA"):
        print(f"    per MFMA: VALU {v.get('SQ_INSTS_VALU', 0) / v['SQ_INSTS_MFMA']:.2f}  LDS {v.get('SQ_INSTS_LDS', 0) / v['SQ_INSTS_MFMA']:.2f}"
              f"  SALU {v.get('SQ_INSTS_SALU', 0) / v['SQ_INSTS_MFMA']:.2f}  VMEM {v.get('SQ_INSTS_VMEM', 0) / v['SQ_INSTS_MFMA']:.2f}")
