"""Representative GEMM / conv launches for rocprofv3 --pmc passes (LDS conflicts, L2 hit rate):
python tools/pmc_cases.py CASE [iters].  Cases: vit_fc1 (bf16 256 phased), vit_wgrad (bf16 256, row-contiguous
operands), r50_c3 (3x3 conv, 128x128 implicit-GEMM core), r50_pw (1x1 conv), r50_dgrad, r50_wgrad."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import ringdp  # noqa: E402

C = ringdp._C
case = sys.argv[1]
it = int(sys.argv[2]) if len(sys.argv) > 2 else 3


def conv_setup(n, h, c, k, r, stride):
    x = torch.randn(n, h, h, c, device="cuda").bfloat16()
    w = torch.randn(k, c, r, r, device="cuda") * 0.05
    krsc, crsk = C.pack_conv_weight(w, c)
    z, _ = C.conv2d_fwd(x, krsc, stride, r // 2, 1, False)
    return x, w, krsc, crsk, z


if case in ("vit_fc1", "vit_wgrad"):
    M, N, K = 25216, 3072, 768
    if case == "vit_fc1":
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = torch.randn(N, K, device="cuda").bfloat16()
        fn = lambda: C.gemm(a, b, M, N, K, K, K, False, False, 1, 0, 0, True, None, 0, None, None)  # noqa: E731
    else:  # dW[n][k] = sum_m dz[m][n] x[m][k]: both operands row-contiguous, split over the tokens
        dz = torch.randn(M, N, device="cuda").bfloat16()
        x = torch.randn(M, K, device="cuda").bfloat16()
        dw = torch.empty(N, K, device="cuda")
        fn = lambda: C.gemm_splitk_f32(dz, x, N, K, M, N, K, True, True, 4, dw)  # noqa: E731
else:
    shape = {"r50_c3": (256, 56, 64, 64, 3, 1), "r50_pw": (256, 56, 64, 256, 1, 1),
             "r50_dgrad": (256, 28, 128, 128, 3, 1), "r50_wgrad": (256, 28, 128, 128, 3, 1)}[case]
    x, w, krsc, crsk, z = conv_setup(*shape)
    n, h, c, k, r, stride = shape
    if case in ("r50_c3", "r50_pw"):
        fn = lambda: C.conv2d_fwd(x, krsc, stride, r // 2, 1, True)  # noqa: E731
    elif case == "r50_dgrad":
        fn = lambda: C.conv2d_dgrad(z, crsk, h, h, stride, r // 2, 1)  # noqa: E731
    else:
        dw = torch.empty_like(w)
        fn = lambda: C.conv2d_wgrad(z, x, dw, stride, r // 2, 1)  # noqa: E731
for _ in range(it):
    fn()
torch.cuda.synchronize()
