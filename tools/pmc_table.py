"""Per-image PMC table from tools/pmc_op.sh outputs (one `<kernel name> {counter: value}` line per pass).

    python tools/pmc_table.py --batch 65536 LABEL=path/to/op.txt:kernel_substring ...

Counters are whole-chip sums over one dispatch (rocprofv3 averages repeated dispatches).  GRBM_GUI_ACTIVE
is summed over the 8 XCDs, so the kernel's wall cycles are GRBM_GUI_ACTIVE / 8 and the MFMA pipe
utilisation is SQ_VALU_MFMA_BUSY_CYCLES / (wall cycles * 256 CUs * 4 SIMDs).
"""
import argparse
import ast


def load(path, pattern):
    out = {}
    with open(path) as f:
        for line in f:
            i = line.find(" {")
            if i < 0 or pattern not in line[:i]:
                continue
            out.update(ast.literal_eval(line[i + 1:].strip()))
    return out


def row(label, c, batch, cus=256):
    g = lambda k: c.get(k, float("nan"))
    wall = g("GRBM_GUI_ACTIVE") / 8
    util = g("SQ_VALU_MFMA_BUSY_CYCLES") / (wall * cus * 4) if wall == wall and wall > 0 else float("nan")
    return (f"| {label} | {g('SQ_INSTS_VALU') / batch:.0f} | {g('SQ_INSTS_MFMA') / batch:.0f} | "
            f"{g('SQ_INSTS_LDS') / batch:.0f} | {g('SQ_LDS_BANK_CONFLICT') / batch:.0f} | "
            f"{g('SQ_WAIT_INST_LDS') / batch:.0f} | {g('FETCH_SIZE') * 1024 / batch / 1000:.1f} | "
            f"{g('WRITE_SIZE') * 1024 / batch / 1000:.1f} | {100 * util:.0f} % |")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("entries", nargs="+", help="LABEL=file:kernel_substring")
    a = ap.parse_args()
    print("| kernel | VALU / img | MFMA / img | LDS / img | LDS bank-conflict cycles / img | "
          "LDS-wait cycles / img | HBM read KB / img | HBM write KB / img | MFMA busy |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for e in a.entries:
        label, rest = e.split("=", 1)
        path, pat = rest.rsplit(":", 1)
        print(row(label, load(path, pat), a.batch))


if __name__ == "__main__":
    main()
