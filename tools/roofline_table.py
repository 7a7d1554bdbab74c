"""Per-kernel roofline table from tools/roofline_convnet.sh output (gpurun_out/roofline/*.csv).

For each ConvNet op group: kernel time (kernel trace), HBM traffic (TCC FETCH_SIZE + WRITE_SIZE, KB),
achieved TB/s, useful TFLOP/s (SURVEY.md §2.6 FLOP counts), LDS bank-conflict cycles per active LDS
cycle.  Only the kernels of the op under test count (the setup forward pass that pmc_run.py runs
first is excluded by taking the last 3 dispatches).

python tools/roofline_table.py [dir] [B] > profiles/r02_convnet_roofline.md
"""
import collections
import csv
import glob
import os
import sys

# useful MFLOP per image of each op group (flop_counter)
OPS = {
    "conv1_fwd": ("conv1_fwd_kernel", 1.08),
    "conv2_fwd": ("conv2_fwd_kernel", 4.46),
    "conv3_fc_fwd": ("conv3_fwd_kernel|fc1_fwd_kernel", 9.44 + 0.04),
    "conv3_fc_bwd": ("conv3_bwd_kernel|fc_bwd_kernel|slab_reduce_kernel", 18.88 + 0.08),
    "conv2_bwd": ("conv2_bwd_kernel|slab_reduce_kernel", 8.92),
    "conv1_wgrad": ("conv1_wgrad_kernel|slab_reduce_kernel", 1.08),
    "conv12_bwd": ("conv12_bwd_kernel|slab_reduce_kernel", 8.92 + 1.08),
}
HBM_TBS = 8.0
BF16_PF = 2.5


def kname(s):
    s = s.replace("(anonymous namespace)", "")
    s = s.split("(")[0]
    return s.split("::")[-1]


def load(d, op, pas):
    f = os.path.join(d, f"{op}_{pas}.csv")
    if not os.path.exists(f):
        return {}
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = kname(r["Kernel_Name"])
        if pas == "time":
            agg[k]["ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        else:
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/roofline"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
    print(f"# ConvNet per-kernel roofline, B={B}, 1x MI355X (rocprofv3; tools/roofline_convnet.sh)\n")
    print("Time: kernel trace. HBM: TCC FETCH_SIZE + WRITE_SIZE (separate passes). FLOP: useful work of the op")
    print(f"(SURVEY.md §2.6), not MFMA padding. Peaks used: {HBM_TBS} TB/s HBM3E, {BF16_PF} PF/s dense bf16.\n")
    print("| op | kernel | us | read MB | write MB | TB/s | % HBM | useful TFLOP/s | % bf16 peak | LDS conflict / active |")
    print("|---|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for op, (pat, mflop) in OPS.items():
        pats = pat.split("|")
        t, fe, wr, lds = (load(d, op, p) for p in ("time", "fetch", "write", "lds"))
        tot_us = 0.0
        for k in t:
            if not any(p in k for p in pats):
                continue
            us = sum(t[k]["ns"][-3:]) / len(t[k]["ns"][-3:]) / 1e3
            rd = sum(fe.get(k, {}).get("FETCH_SIZE", [0])[-3:]) / 3 / 1024
            wt = sum(wr.get(k, {}).get("WRITE_SIZE", [0])[-3:]) / 3 / 1024
            conf = lds.get(k, {}).get("SQ_LDS_BANK_CONFLICT", [0])
            act = lds.get(k, {}).get("SQ_ACTIVE_INST_LDS", [0])
            ratio = (sum(conf[-3:]) / max(1.0, sum(act[-3:]))) if act else 0.0
            tbs = (rd + wt) / 1e6 / (us * 1e-6)
            main_k = pats[0] in k
            tf = (mflop * 1e6 * B / (us * 1e-6) / 1e12) if main_k else None
            tot_us += us
            print(f"| {op} | {k[:40]} | {us:.1f} | {rd:.0f} | {wt:.0f} | {tbs:.2f} | {100 * tbs / HBM_TBS:.0f} | "
                  f"{'' if tf is None else f'{tf:.0f}'} | {'' if tf is None else f'{100 * tf / 1000 / BF16_PF:.0f}'} | "
                  f"{ratio:.2f} |")
        if tot_us:
            print(f"| {op} | **group total** | **{tot_us:.1f}** | | | | | **{mflop * 1e6 * B / (tot_us * 1e-6) / 1e12:.0f}** | | |")


if __name__ == "__main__":
    main()
