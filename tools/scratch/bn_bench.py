"""Bandwidth of the NHWC batch-norm kernels (ResNet-50 shapes, B=256): bn_fwd_train (apply + ReLU),
bn_bwd (reduce + apply) -> us and effective TB/s over the bytes each must move."""
import json
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters * 1000.0


def case(n, h, c, res):
    z = torch.randn(n, h, h, c, device="cuda").bfloat16()
    r = torch.randn_like(z) if res else None
    g, bt = torch.ones(c, device="cuda"), torch.zeros(c, device="cuda")
    rm, rv = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
    zf = z.float().view(-1, c)
    sums = torch.stack([zf.sum(0), (zf * zf).sum(0)]).contiguous()
    y, save = C.bn_fwd_train(z, sums, g, bt, rm, rv, 1e-5, 0.1, r, True)
    dy = torch.randn_like(z)
    dg, db = torch.zeros(c, device="cuda"), torch.zeros(c, device="cuda")
    tf = timeit(lambda: C.bn_fwd_train(z, sums, g, bt, rm, rv, 1e-5, 0.1, r, True))
    tb = timeit(lambda: C.bn_bwd(dy, y, z, save, g, True, dg, db))
    nb = z.numel() * 2
    return {"shape": f"{n}x{h}x{h}x{c} res={res}", "fwd_us": round(tf, 1), "fwd_TBs": round((2 + res) * nb / tf / 1e6, 2),
            "bwd_us": round(tb, 1), "bwd_TBs": round(7 * nb / tb / 1e6, 2)}


if __name__ == "__main__":
    for args in [(256, 56, 64, 0), (256, 56, 256, 1), (256, 28, 512, 1), (256, 14, 1024, 1), (256, 7, 2048, 1),
                 (256, 112, 64, 0)]:
        print(json.dumps(case(*args)), flush=True)
