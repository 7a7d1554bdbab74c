"""Error pattern of the fp32 conv3 scatter dgrad against fp64 (which images / channels / positions)."""
import sys
import torch
sys.path.insert(0, ".")
from ringdp._native import C

for B in (512, 600, 700, 1024):
    g = torch.Generator(device="cuda").manual_seed(B)
    w = torch.randn(128, 64, 3, 3, device="cuda", generator=g) * 0.1
    dz = torch.randn(B, 128, 8, 8, device="cuda", generator=g)
    dx = C.f32_conv_dgrad(dz, w, 10, 10, 0)
    ref = torch.nn.grad.conv2d_input((B, 64, 10, 10), w.double(), dz.double()).float()
    err = (dx - ref).abs()
    bad = err > 1e-3
    print("B", B, "max err", float(err.max()), "bad", int(bad.sum()), "of", err.numel(), flush=True)
    if bad.any():
        idx = bad.nonzero()
        print("  images", sorted(set(idx[:, 0].tolist()))[:20], "n", len(set(idx[:, 0].tolist())))
        print("  channels", sorted(set(idx[:, 1].tolist())))
        print("  rows", sorted(set(idx[:, 2].tolist())), "cols", sorted(set(idx[:, 3].tolist())))
        b0 = int(idx[0, 0])
        print("  sample", dx[b0, :2, :3, :3].tolist(), ref[b0, :2, :3, :3].tolist())
