"""hipBLASLt e4m3 path vs ringdp's fp8 kernels (numerics and timing) on the ViT-B/16 fp8 GEMMs."""
import json
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters * 1000


def q(t):
    return t.to(torch.float8_e4m3fn).view(torch.uint8)


def main():
    torch.manual_seed(0)
    sa = torch.tensor([0.5], device="cuda")
    sb = torch.tensor([0.25], device="cuda")
    for (M, N, K) in [(25216, 2304, 768), (25216, 768, 768), (25216, 3072, 768), (25216, 768, 3072),
                      (768, 768, 25216), (3072, 768, 25216)]:
        A = torch.randn(M, K, device="cuda") * 2
        B = torch.randn(N, K, device="cuda") * 2
        Aq, Bq = q(A), q(B)
        bias = torch.randn(N, device="cuda")
        ref = (Aq.view(torch.float8_e4m3fn).float() @ Bq.view(torch.float8_e4m3fn).float().t()) * 0.125
        row = {"shape": f"{M}x{N}x{K}"}
        for be in ("auto", "ringdp"):
            C.set_gemm_backend(be)
            if K > 20000:  # weight-gradient shape: fp32 output through the split-K entry
                out = torch.empty(M, N, device="cuda")
                f = lambda: C.gemm_fp8_splitk_f32(Aq, Bq, sa, sb, M, N, K, 8, out)
                f()
                torch.cuda.synchronize()
                got = out
            else:
                f = lambda: C.gemm_fp8(Aq, Bq, sa, sb, M, N, K, True, bias)
                got = f().float()
                ref_b = ref + bias
            torch.cuda.synchronize()
            r = ref if K > 20000 else ref_b
            row[f"{be}_relerr"] = float((got - r).abs().max() / r.abs().max())
            us = timeit(f)
            row[f"{be}_us"] = round(us, 1)
            row[f"{be}_TF"] = round(2 * M * N * K / us / 1e6, 1)
        print(json.dumps(row), flush=True)
    C.set_gemm_backend("auto")


if __name__ == "__main__":
    main()
