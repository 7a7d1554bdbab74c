"""Comm/compute overlap from a rocprofv3 kernel trace (``--kernel-trace --output-format csv``).

    python tools/overlap_trace.py run_kernel_trace.csv [--comm xgmi_kernel<float] [--last-ms 200]

Comm kernels are those whose name contains ``--comm`` (the bucket collectives: ringdp's xgmi kernels or
RCCL's); compute kernels are the others on the queue that runs the most kernels (the captured step).  For the comm kernels that start in the
last ``--last-ms`` of the trace it reports how much of each one's duration ran while a compute kernel was
running (the union of compute intervals), i.e. how much of the collective was hidden behind backward.
"""
import argparse
import csv


def union(intervals):
    out = []
    for s, e in sorted(intervals):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def covered(s, e, merged):
    t = 0
    for a, b in merged:
        if b <= s:
            continue
        if a >= e:
            break
        t += min(b, e) - max(a, s)
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--comm", default="xgmi_kernel<float")
    ap.add_argument("--last-ms", type=float, default=200.0)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], (r["Queue_Id"], r["Stream_Id"]))
          for r in rows]
    t_end = max(k[1] for k in ks)
    t0 = t_end - int(a.last_ms * 1e6)
    # the compute queue: the one that runs most kernels (the captured step); comm kernels may run there too
    # (buckets captured inline) or on the process group's comm queue
    counts = {}
    for k in ks:
        counts[k[3]] = counts.get(k[3], 0) + 1
    cq = max(counts, key=counts.get)
    comm = [k for k in ks if a.comm in k[2] and k[0] >= t0]
    comp = union([(k[0], k[1]) for k in ks if a.comm not in k[2] and k[3] == cq and k[1] >= t0])
    side = [k for k in comm if k[3] != cq]
    tot = sum(e - s for s, e, _, _ in comm)
    hid = sum(covered(s, e, comp) for s, e, _, _ in comm)
    tot_side = sum(e - s for s, e, _, _ in side)
    print("| trace | comm kernels (on the comm queue) | comm us (on the comm queue) | overlapped with compute us | "
          "hidden |")
    print("|---|---:|---:|---:|---:|")
    print(f"| {a.trace} | {len(comm)} ({len(side)}) | {tot / 1e3:.1f} ({tot_side / 1e3:.1f}) | {hid / 1e3:.1f} | "
          f"{100.0 * hid / max(tot, 1):.0f} % |")
    if side:  # one comm-queue collective in context: the compute kernels running while it ran
        s, e, name, q = side[len(side) // 2]
        print(f"\nsample collective {name[:60]} on queue/stream {q}: {s - t0} .. {e - t0} ns "
              f"({(e - s) / 1e3:.1f} us); compute kernels overlapping it:")
        for ks_, ke, kn, kq in ks:
            if a.comm not in kn and kq == cq and ke > s and ks_ < e:
                print(f"  {ks_ - t0:>12} .. {ke - t0:>12}  {kn[:90]}")


if __name__ == "__main__":
    main()
