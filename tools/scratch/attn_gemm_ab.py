"""A/B of ViT-B/16's unfused attention-backward GEMMs (dQ = dS K, dK = dS^T Q, dV = P^T dO; batch
B*H = 1536 heads, Tp = 208, Dh = 64): ringdp's checked 128x128 core vs hipBLASLt (RINGDP_BLASLT_ROW=2).
python tools/attn_gemm_ab.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C
BH, Tp, Dh = 1536, 208, 64


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters * 1000.0


def main():
    torch.manual_seed(0)
    ds = torch.randn(BH, Tp, Tp, device="cuda").bfloat16()
    q = torch.randn(BH, Tp, Dh, device="cuda").bfloat16()
    cases = {
        "dq = ds k": lambda: C.gemm(ds, q, Tp, Dh, Tp, Tp, Dh, False, True, BH, Tp * Tp, Tp * Dh, True),
        "dk = ds^T q": lambda: C.gemm(ds, q, Tp, Dh, Tp, Tp, Dh, True, True, BH, Tp * Tp, Tp * Dh, True),
    }
    ref = {"dq = ds k": torch.bmm(ds.float(), q.float()), "dk = ds^T q": torch.bmm(ds.float().transpose(1, 2), q.float())}
    for name, f in cases.items():
        out = f().view(BH, Tp, Dh).float()
        err = float((out - ref[name]).abs().max() / ref[name].abs().max())
        print(json.dumps({"case": name, "us": round(timeit(f), 1), "err": err}), flush=True)


if __name__ == "__main__":
    main()
