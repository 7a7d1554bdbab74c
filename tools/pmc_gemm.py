"""One dense GEMM shape, repeated, for rocprofv3 --pmc passes: python tools/pmc_gemm.py M N K [iters] [fp8]"""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import ringdp  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
it = int(sys.argv[4]) if len(sys.argv) > 4 else 3
fp8 = "fp8" in sys.argv[5:]
if fp8:
    a = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn).view(torch.uint8)
    b = torch.randn(N, K, device="cuda").to(torch.float8_e4m3fn).view(torch.uint8)
    one = torch.ones(1, device="cuda")
else:
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(N, K, device="cuda").bfloat16()
for _ in range(it):
    if fp8:
        ringdp._C.gemm_fp8(a, b, one, one, M, N, K, True)
    else:
        ringdp._C.gemm(a, b, M, N, K, K, K, False, False, 1, 0, 0, True, None, 0, None, None)
torch.cuda.synchronize()
