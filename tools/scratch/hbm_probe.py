"""HBM write / read / copy bandwidth probe on one MI355X (calibrates the ConvNet roofline's write side).
python tools/hbm_probe.py"""
import json

import torch


def t(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters * 1e-3


for mb in (256, 512, 1024, 4096):
    n = mb * 2**20 // 4
    x = torch.empty(n, device="cuda")
    y = torch.empty(n, device="cuda")
    x.fill_(1.0)
    w = t(lambda: x.fill_(0.5))
    r = t(lambda: x.sum())
    c = t(lambda: y.copy_(x))
    print(json.dumps({"MB": mb, "write_TBs": round(mb * 2**20 / w / 1e12, 2), "read_TBs": round(mb * 2**20 / r / 1e12, 2),
                      "copy_TBs(r+w)": round(2 * mb * 2**20 / c / 1e12, 2)}), flush=True)
