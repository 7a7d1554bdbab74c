"""Per-layer table of the fp32 ConvNet kernels from a rocprofv3 kernel trace (avg us per call)."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if "kern::" not in n or "synth" in n:
        continue
    m = re.search(r"gemm_f32_kernel<(\d), (\d), [^,]*::(\w+), [^,]*::(\w+)", n)
    key = f"gemm{m.group(1)}{m.group(2)} {m.group(3)}" if m else n.split("(")[0].split("::")[-1]
    key += f" grid=({r['Grid_Size_X']},{r['Grid_Size_Y']},{r['Grid_Size_Z']})"
    d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0.0
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]) / len(kv[1])):
    a = sum(v) / len(v)
    print(f"{a:9.0f} us  x{len(v):3d}  {k}")
