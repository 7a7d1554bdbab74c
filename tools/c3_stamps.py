"""Phase timing of the conv3 backward v2 dgrad role from a -DRINGDP_C3V_STAMP build (s_memtime stamps of
workgroup 0): RINGDP_EXT_PATH=<stamp build> python tools/c3_stamps.py [B]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_run  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
fns = pmc_run.build_ops(B)
for _ in range(3):
    fns["conv3_fc_bwd"]()
torch.cuda.synchronize()
C = pmc_run.C
st = C.cn_debug_stamps()
assert st is not None and st.numel(), "not a stamp build"
names = ["top", "barA", "dmawait", "expand", "barB", "pass0", "x6", "pass1", "x8"]
out = {}
for w in range(4):
    rows = []
    for img in range(2, 15):  # steady state
        t = st[w, img].tolist()
        tn = st[w, img + 1, 0].item()
        d = {"barA": t[1] - t[0], "dmawait": t[2] - t[1], "expand": t[9] - t[2], "codes_dma": t[10] - t[9],
             "load_pre": t[3] - t[10], "barB": t[4] - t[3], "pass0": t[5] - t[4], "pass1": t[7] - t[5]}
        d["tail"] = tn - t[7]
        d["total"] = tn - t[0]
        rows.append(d)
    out[f"wave{w}"] = {k: round(sum(r[k] for r in rows) / len(rows)) for k in rows[0]}
print(json.dumps(out, indent=1))
