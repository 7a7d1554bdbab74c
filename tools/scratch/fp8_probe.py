"""Probe the fp8 (e4m3) MFMA GEMM path against exact references (integer and random data)."""
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C


def check(M, N, K, rnd):
    torch.manual_seed(0)
    one = torch.ones(1, device="cuda")
    if rnd:
        A = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn)
        B = torch.randn(N, K, device="cuda").to(torch.float8_e4m3fn)
    else:
        A = torch.randint(-3, 4, (M, K), device="cuda").float().to(torch.float8_e4m3fn)
        B = torch.randint(-3, 4, (N, K), device="cuda").float().to(torch.float8_e4m3fn)
    out = C.gemm_fp8(A.view(torch.uint8).contiguous(), B.view(torch.uint8).contiguous(), one, one, M, N, K, False)
    ref = (A.double() @ B.double().t())
    bf = C.gemm(A.float().bfloat16(), B.float().bfloat16(), M, N, K, K, K, False, False, 1, 0, 0, False).view(M, N)
    e = (out.double() - ref).abs().max() / ref.abs().max()
    eb = (bf.double() - ref).abs().max() / ref.abs().max()
    print(f"M{M} N{N} K{K} rnd={rnd}: fp8 rel {float(e):.2e}  bf16-core rel {float(eb):.2e}", flush=True)


for args in [(128, 128, 128, False), (128, 128, 768, False), (320, 272, 768, False), (128, 128, 128, True),
             (128, 128, 768, True), (320, 272, 768, True)]:
    check(*args)

# large-magnitude operands (as after per-tensor scaling to the e4m3 range)
for mag in (1.0, 30.0, 100.0):
    torch.manual_seed(1)
    M, N, K = 320, 272, 768
    one = torch.ones(1, device="cuda")
    A = (torch.randn(M, K, device="cuda") * mag).clamp(-448, 448).to(torch.float8_e4m3fn)
    B = (torch.randn(N, K, device="cuda") * mag).clamp(-448, 448).to(torch.float8_e4m3fn)
    out = C.gemm_fp8(A.view(torch.uint8).contiguous(), B.view(torch.uint8).contiguous(), one, one, M, N, K, False)
    ref = A.double() @ B.double().t()
    print(f"mag {mag}: rel {float((out.double() - ref).abs().max() / ref.abs().max()):.2e}", flush=True)
