"""One dense GEMM shape, repeated, for rocprofv3 --pmc passes: python tools/pmc_gemm.py M N K [iters]"""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import ringdp  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
it = int(sys.argv[4]) if len(sys.argv) > 4 else 3
a = torch.randn(M, K, device="cuda").bfloat16()
b = torch.randn(N, K, device="cuda").bfloat16()
for _ in range(it):
    ringdp._C.gemm(a, b, M, N, K, K, K, False, False, 1, 0, 0, True, None, 0, None, None)
torch.cuda.synchronize()
