"""A/B of the ViT-B/16 weight-gradient GEMMs (dW = dz^T x over 25216 token rows, both operands
row-contiguous): ringdp's 128x128 split-K core vs the 256x256 transposed-read kernel, with the split
counts each path picks.  python tools/wgrad256_ab.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402
from ringdp.ops.transformer import _splits  # noqa: E402

C = ringdp._C
T = 25216
SHAPES = [(2304, 768, "qkv"), (768, 768, "proj"), (3072, 768, "fc1"), (768, 3072, "fc2")]


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
    for M, N, note in SHAPES:
        dz = (torch.randn(T, M, device="cuda") * 0.5).bfloat16()
        x = (torch.randn(T, N, device="cuda") * 0.5).bfloat16()
        out = torch.empty(M, N, device="cuda")
        res = {"shape": f"{M}x{N}x{T}", "note": note}
        ref = dz.float().t() @ x.float()
        for mode in (128, 256, 0):
            C.set_bf16_tile_mode(mode)
            f = lambda: C.gemm_splitk_f32(dz, x, M, N, T, M, N, True, True, _splits(T, M, N), out)
            f()
            res[f"err{mode}"] = float((out - ref).abs().max() / ref.abs().max())
            us = timeit(f)
            res[f"k{mode}_us"] = round(us, 1)
            res[f"k{mode}_TF"] = round(2 * M * N * T / us / 1e6, 1)
        C.set_bf16_tile_mode(0)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
