"""hipBLASLt backend vs ringdp's GEMM kernels on every epilogue the ops use, and timing on the ViT /
ResNet plain-GEMM shapes.  python tools/blaslt_check.py"""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C


def run(backend, *args, **kw):
    C.set_gemm_backend(backend)
    out = C.gemm(*args, **kw)
    torch.cuda.synchronize()
    return out


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


def main():
    torch.manual_seed(0)
    M, N, K = 1000, 776, 512
    A = torch.randn(M, K, device="cuda").bfloat16()
    B = torch.randn(N, K, device="cuda").bfloat16()
    bias = torch.randn(N, device="cuda")
    res = torch.randn(M, N, device="cuda").bfloat16()
    ref = A.float() @ B.float().t()
    cases = {
        "plain_f32": dict(args=(A, B, M, N, K, K, K, False, False, 1, 0, 0, False)),
        "bias_bf16": dict(args=(A, B, M, N, K, K, K, False, False, 1, 0, 0, True, bias)),
        "residual": dict(args=(A, B, M, N, K, K, K, False, False, 1, 0, 0, True, bias, 0, res)),
    }
    for name, c in cases.items():
        o1 = run("auto", *c["args"]).float().view(M, N)
        o2 = run("ringdp", *c["args"]).float().view(M, N)
        print(json.dumps({"case": name, "max_diff": float((o1 - o2).abs().max()), "ref_max": float(ref.abs().max())}))
    # GELU with pre-activation: which GELU does the library apply?
    pre1 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    pre2 = torch.empty_like(pre1)
    g1 = run("auto", A, B, M, N, K, K, K, False, False, 1, 0, 0, False, bias, 2, None, pre1).view(M, N)
    g2 = run("ringdp", A, B, M, N, K, K, K, False, False, 1, 0, 0, False, bias, 2, None, pre2).view(M, N)
    z = ref + bias
    erf = 0.5 * z * (1 + torch.erf(z / math.sqrt(2)))
    tanh = 0.5 * z * (1 + torch.tanh(math.sqrt(2 / math.pi) * (z + 0.044715 * z ** 3)))
    print(json.dumps({"case": "gelu_aux", "lt_vs_erf": float((g1 - erf).abs().max()), "lt_vs_tanh": float((g1 - tanh).abs().max()),
                      "ringdp_vs_erf": float((g2 - erf).abs().max()), "preact_diff": float((pre1.float() - pre2.float()).abs().max())}))
    # transposed layouts (dgrad: B row-contiguous; wgrad: both row-contiguous, fp32 out via split-K entry)
    Bt = B.t().contiguous()  # [K][N]
    o1 = run("auto", A, Bt, M, N, K, K, N, False, True, 1, 0, 0, False).view(M, N)
    print(json.dumps({"case": "b_row", "max_diff": float((o1 - ref).abs().max())}))
    At = A.t().contiguous()
    out = torch.empty(M, N, device="cuda")
    C.set_gemm_backend("auto")
    C.gemm_splitk_f32(At, Bt, M, N, K, M, N, True, True, 4, out)
    torch.cuda.synchronize()
    print(json.dumps({"case": "splitk_rowrow", "max_diff": float((out - ref).abs().max())}))
    # timing on the ViT shapes (forward K-contiguous, dgrad B row, wgrad both row)
    for (m, n, k) in [(25216, 2304, 768), (25216, 768, 768), (25216, 3072, 768), (25216, 768, 3072)]:
        a = torch.randn(m, k, device="cuda").bfloat16()
        w = torch.randn(n, k, device="cuda").bfloat16()
        dz = torch.randn(m, n, device="cuda").bfloat16()
        row = {"shape": f"{m}x{n}x{k}"}
        for be in ("auto", "ringdp"):
            C.set_gemm_backend(be)
            row[f"fwd_{be}_us"] = round(timeit(lambda: C.gemm(a, w, m, n, k, k, k, False, False, 1, 0, 0, True)), 1)
            row[f"dgrad_{be}_us"] = round(timeit(lambda: C.gemm(dz, w, m, k, n, n, k, False, True)), 1)
            dw = torch.empty(n, k, device="cuda")
            row[f"wgrad_{be}_us"] = round(timeit(lambda: C.gemm_splitk_f32(dz, a, n, k, m, n, k, True, True, 8, dw)), 1)
        print(json.dumps(row), flush=True)
    C.set_gemm_backend("auto")


if __name__ == "__main__":
    main()
