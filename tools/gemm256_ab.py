"""A/B of the bf16 GEMM kernels on K-contiguous shapes: 128x128 core vs the 256x256 LDS-DMA kernel vs
torch.matmul (hipBLASLt), plus a correctness check of the 256 path against an fp32 reference.
python tools/gemm256_ab.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C

SHAPES = [  # (M, N, K, note)
    (25216, 2304, 768, "vit qkv fwd"), (25216, 768, 768, "vit proj fwd"), (25216, 3072, 768, "vit fc1 fwd"),
    (25216, 768, 3072, "vit fc2 fwd"), (4096, 4096, 4096, "square"), (8192, 8192, 8192, "square"),
    (802816, 64, 256, "r50 1x1 56x56 256->64"), (802816, 256, 64, "r50 1x1 56x56 64->256"),
    (200704, 512, 128, "r50 1x1 28x28 128->512"), (200704, 128, 512, "r50 1x1 28x28 512->128"),
    (50176, 1024, 256, "r50 1x1 14x14 256->1024"), (50176, 256, 1024, "r50 1x1 14x14 1024->256"),
    (12544, 2048, 512, "r50 1x1 7x7 512->2048"), (12544, 512, 2048, "r50 1x1 7x7 2048->512"),
]


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
    for M, N, K, note in SHAPES:
        A = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
        B = (torch.randn(N, K, device="cuda") * 0.5).bfloat16()
        bias = torch.randn(N, device="cuda")
        res = {"shape": f"{M}x{N}x{K}", "note": note}
        outs = {}
        for mode in (128, 256):
            C.set_bf16_tile_mode(mode)
            f = lambda: C.gemm(A, B, M, N, K, K, K, False, False, 1, 0, 0, True, bias)
            outs[mode] = f().view(M, N).float()
            us = timeit(f)
            res[f"k{mode}_us"] = round(us, 1)
            res[f"k{mode}_TF"] = round(2 * M * N * K / us / 1e6, 1)
        C.set_bf16_tile_mode(0)
        us = timeit(lambda: torch.matmul(A, B.t()))
        res["hipblaslt_us"] = round(us, 1)
        res["hipblaslt_TF"] = round(2 * M * N * K / us / 1e6, 1)
        rows = slice(0, min(M, 4096))
        ref = (A[rows].float() @ B.float().t()) + bias
        res["err256"] = float((outs[256][rows] - ref).abs().max() / ref.abs().max())
        res["err128"] = float((outs[128][rows] - ref).abs().max() / ref.abs().max())
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
