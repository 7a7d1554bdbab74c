"""Kernel table (markdown) from a rocprofv3 --kernel-trace database (run_results.db):
python tools/rocpd_table.py <dir-with-run_results.db> [out.md]"""
import glob
import os
import sqlite3
import sys


def short(n):
    for pre in ("void ringdp::kern::(anonymous namespace)::", "ringdp::kern::(anonymous namespace)::",
                "void (anonymous namespace)::", "void at::native::"):
        if n.startswith(pre):
            n = n[len(pre):]
    if n.startswith("_ZN6ringdp4kern12_GLOBAL__N_1"):
        import re
        m = re.match(r"_ZN6ringdp4kern12_GLOBAL__N_1\d+([A-Za-z0-9_]+?)E", n)
        n = m.group(1) if m else n
    return n.split("(")[0][:70]


def main():
    d = sys.argv[1]
    db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, count(*), avg(end-start)/1000.0, min(end-start)/1000.0, "
                          "max(end-start)/1000.0 from kernels group by name order by sum(end-start) desc"))
    tot = sum(r[1] * r[2] for r in rows)
    out = ["| kernel | calls | avg us | min us | max us | % time |", "|---|---:|---:|---:|---:|---:|"]
    for r in rows:
        out.append(f"| {short(r[0])} | {r[1]} | {r[2]:.1f} | {r[3]:.1f} | {r[4]:.1f} | {100 * r[1] * r[2] / tot:.1f} |")
    text = "\n".join(out) + "\n"
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
