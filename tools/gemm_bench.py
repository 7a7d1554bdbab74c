"""Throughput of the generic MFMA GEMM core: dense layouts and ResNet-50 conv shapes (B=256)."""
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
    return a.elapsed_time(b) / iters * 1000.0  # us


def dense(M, N, K, a_row=False, b_row=False):
    A = torch.randn(K * M, device="cuda").bfloat16()
    B = torch.randn(K * N, device="cuda").bfloat16()
    lda = M if a_row else K
    ldb = N if b_row else K
    us = timeit(lambda: C.gemm(A, B, M, N, K, lda, ldb, a_row, b_row, 1, 0, 0, True))
    return {"shape": f"dense {M}x{N}x{K} a_row={a_row} b_row={b_row}", "us": round(us, 1),
            "TFLOPs": round(2 * M * N * K / us / 1e6, 1)}


def dense_fp8(M, N, K):
    A = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn).view(torch.uint8)
    B = torch.randn(N, K, device="cuda").to(torch.float8_e4m3fn).view(torch.uint8)
    one = torch.ones(1, device="cuda")
    us = timeit(lambda: C.gemm_fp8(A, B, one, one, M, N, K, True))
    return {"shape": f"fp8 dense {M}x{N}x{K}", "us": round(us, 1), "TFLOPs": round(2 * M * N * K / us / 1e6, 1)}


def conv(n, h, c, k, r, stride):
    pad = r // 2
    x = torch.randn(n, h, h, c, device="cuda").bfloat16()
    w = torch.randn(k, c, r, r, device="cuda") * 0.05
    krsc, crsk = C.pack_conv_weight(w, c)
    z, _ = C.conv2d_fwd(x, krsc, stride, pad, 1, False)
    p = z.shape[1]
    flops = 2 * n * p * p * k * c * r * r
    f = timeit(lambda: C.conv2d_fwd(x, krsc, stride, pad, 1, False))
    fs = timeit(lambda: C.conv2d_fwd(x, krsc, stride, pad, 1, True))
    d = timeit(lambda: C.conv2d_dgrad(z, crsk, h, h, stride, pad, 1))
    dw = torch.empty_like(w)
    wg = timeit(lambda: C.conv2d_wgrad(z, x, dw, stride, pad, 1))
    return {"shape": f"conv n{n} {h}x{h} c{c}->k{k} r{r} s{stride}",
            "fwd": [round(f, 1), round(flops / f / 1e6, 1)], "fwd+stats_us": round(fs, 1),
            "dgrad": [round(d, 1), round(flops / d / 1e6, 1)], "wgrad": [round(wg, 1), round(flops / wg / 1e6, 1)]}


def attention(BH=1536, Tp=208, Dh=64):
    """ViT-B/16 attention batched GEMMs (B=128 x 12 heads, Tp=208 padded tokens, head dim 64)."""
    q = torch.randn(BH * Tp * Dh, device="cuda").bfloat16()
    k = torch.randn(BH * Tp * Dh, device="cuda").bfloat16()
    p = torch.randn(BH * Tp * Tp, device="cuda").bfloat16()
    res = {}
    res["QK^T"] = timeit(lambda: C.gemm(q, k, Tp, Tp, Dh, Dh, Dh, False, False, BH, Tp * Dh, Tp * Dh, False))
    res["PV"] = timeit(lambda: C.gemm(p, k, Tp, Dh, Tp, Tp, Dh, False, True, BH, Tp * Tp, Tp * Dh, True))
    res["dS^T Q"] = timeit(lambda: C.gemm(p, q, Tp, Dh, Tp, Tp, Dh, True, True, BH, Tp * Tp, Tp * Dh, True))
    return {"shape": f"attention BH{BH} Tp{Tp} Dh{Dh}", **{n: round(v, 1) for n, v in res.items()}}


def vit_fp8_layer(M=25216, D=768, F=3072):
    """The 12 fp8 GEMMs of one ViT-B/16 block as ringdp/ops/transformer.py issues them (us each)."""
    from ringdp.ops.transformer import _splits
    one = torch.ones(1, device="cuda")
    q = lambda r, c: torch.randn(r, c, device="cuda").to(torch.float8_e4m3fn).view(torch.uint8)
    res = {}
    for name, n_out, k_in in (("qkv", 3 * D, D), ("proj", D, D), ("fc1", F, D), ("fc2", D, F)):
        x, w, wt, dz = q(M, k_in), q(n_out, k_in), q(k_in, n_out), q(M, n_out)
        xt, dzt = q(k_in, M), q(n_out, M)
        dw = torch.empty(n_out, k_in, device="cuda")
        f = timeit(lambda: C.gemm_fp8(x, w, one, one, M, n_out, k_in, True))
        d = timeit(lambda: C.gemm_fp8(dz, wt, one, one, M, k_in, n_out, True))
        sp = _splits(M, n_out, k_in)
        g = timeit(lambda: C.gemm_fp8_splitk_f32(dzt, xt, one, one, n_out, k_in, M, sp, dw))
        fl = 2 * M * n_out * k_in / 1e6
        res[name] = {"fwd": [round(f, 1), round(fl / f, 0)], "dgrad": [round(d, 1), round(fl / d, 0)],
                     "wgrad": [round(g, 1), round(fl / g, 0)], "splits": sp}
    return res


if __name__ == "__main__":
    out = []
    if "--vit-fp8" in sys.argv:
        print(json.dumps(vit_fp8_layer()), flush=True)
        for args in [(4096, 4096, 4096), (8192, 8192, 8192)]:
            print(json.dumps(dense_fp8(*args)), flush=True)
        sys.exit(0)
    if "--attention" in sys.argv:
        print(json.dumps(attention()), flush=True)
        sys.exit(0)
    for args in [(4096, 4096, 4096), (4096, 4096, 4096, True, False), (4096, 4096, 4096, False, True),
                 (4096, 4096, 4096, True, True), (8192, 768, 3072)]:
        out.append(dense(*args))
        print(json.dumps(out[-1]), flush=True)
    for args in [(4096, 4096, 4096), (8192, 8192, 8192), (25216, 3072, 768), (25216, 768, 3072)]:
        out.append(dense_fp8(*args))
        print(json.dumps(out[-1]), flush=True)
    for args in [(8192, 8192, 8192), (25216, 3072, 768), (25216, 768, 3072), (25216, 2304, 768)]:
        out.append(dense(*args))
        print(json.dumps(out[-1]), flush=True)
    for args in [(256, 56, 64, 64, 1, 1), (256, 56, 64, 64, 3, 1), (256, 56, 64, 256, 1, 1), (256, 56, 256, 64, 1, 1),
                 (256, 28, 128, 128, 3, 1), (256, 14, 256, 256, 3, 1), (256, 7, 512, 512, 3, 1),
                 (256, 14, 1024, 256, 1, 1), (256, 224, 8, 64, 7, 2)]:
        out.append(conv(*args))
        print(json.dumps(out[-1]), flush=True)

