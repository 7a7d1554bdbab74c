"""Summarise a rocprofv3 kernel trace of N graph-replayed steps: per-step wall, kernel busy time (union of
kernel intervals), gaps, and per-kernel averages.  python tools/timeline.py trace.csv [steps]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    # the timed steps are the last `steps` occurrences of the optimizer kernel
    sgd = [i for i, e in enumerate(ev) if "sgd_flat" in e[2]]
    last = sgd[-steps:]
    lo = ev[sgd[-steps - 1]][1] if len(sgd) > steps else ev[0][0]
    hi = ev[last[-1]][1]
    win = [e for e in ev if e[0] >= lo and e[1] <= hi]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = hi - lo
    print(f"window {wall / 1e3 / steps:.1f} us/step, kernels busy {busy / 1e3 / steps:.1f} us/step, "
          f"idle {(wall - busy) / 1e3 / steps:.1f} us/step, {len(win) / steps:.1f} kernels/step")
    agg = collections.defaultdict(list)
    for s, e, n in win:
        k = n.replace("(anonymous namespace)", "").split("(")[0].split("::")[-1][:60]
        agg[k].append(e - s)
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{sum(v) / 1e3 / steps:9.1f} us/step  {len(v) / steps:4.1f}x  avg {sum(v) / len(v) / 1e3:8.1f} us  {k}")


if __name__ == "__main__":
    main()
