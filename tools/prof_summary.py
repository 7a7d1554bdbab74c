"""Summarise a rocprofv3 ``*_kernel_stats.csv`` into a markdown table (for profiles/)."""
import csv
import re
import sys


def short(name: str) -> str:
    if "gemm_kernel<" in name:  # keep the loader pair: the instantiations are different convolutions
        args = name.split("gemm_kernel<", 1)[1].split(">(", 1)[0]
        args = re.sub(r"ringdp::kern::|\(anonymous namespace\)::", "", args)
        return f"gemm_kernel<{args}>"
    m = re.search(r"(\w+_kernel)(?:<[^>]*>)?", name.replace("EEv", "E"))
    if m:
        k = m.group(1)
        k = re.sub(r"^.*_GLOBAL__N_\d+", "", k)
        tm = re.search(r"_kernel<(\w+)>", name)
        return k + (f"<{tm.group(1)}>" if tm else "")
    return name[:60]


def main(path, top=20):
    rows = list(csv.DictReader(open(path)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print("| kernel | calls | avg us | min us | max us | % time |")
    print("|---|---:|---:|---:|---:|---:|")
    for r in rows[:top]:
        print(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
              f"{float(r['MinNs'])/1e3:.1f} | {float(r['MaxNs'])/1e3:.1f} | {100*float(r['TotalDurationNs'])/total:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
