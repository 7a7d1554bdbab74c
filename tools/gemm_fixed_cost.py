"""Per-block fixed cost of the 256x256 GEMM: time M x N x K for growing K (operands aliased to one row,
lda = ldb = 0, so every load hits on-chip caches) and fit t = a + b K.  Per-block fixed cost ~ a /
rounds.  Output bf16 (8-B stores) vs fp32 (16-B stores) separates the store path.
python tools/gemm_fixed_cost.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C


def timeit(fn, iters=30, warm=5):
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


def reference(M, N):
    """What the memory system and the library do on the same output: pure write, copy, hipBLASLt."""
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    out2 = torch.empty_like(out)
    nb = out.numel() * 2
    res = {"M": M, "N": N, "fill_TBps": round(nb / timeit(lambda: out.fill_(0.5)) / 1e6, 2),
           "copy_TBps_rw": round(2 * nb / timeit(lambda: out2.copy_(out)) / 1e6, 2)}
    for K in (64, 768):
        A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        res[f"torch_matmul_K{K}_us"] = round(timeit(lambda: torch.matmul(A, B.t())), 1)
    print(json.dumps(res), flush=True)


def main():
    for M, N in ((25216, 2304), (4096, 4096)):
        reference(M, N)
    C.set_bf16_tile_mode(256)
    for M, N in ((25216, 2304), (4096, 4096)):
        for out_bf16, wide in ((True, 2), (True, 12), (True, 1)):
            C.set_gemm_wide_store(wide)
            pts = []
            for K in (64, 128, 256, 512, 768, 1536, 3072):
                A = (torch.rand(1, K, device="cuda") * 2 - 1).bfloat16()
                B = (torch.rand(1, K, device="cuda") * 2 - 1).bfloat16()
                out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16 if out_bf16 else torch.float32)
                f = lambda: C.gemm(A, B, M, N, K, 0, 0, False, False, 1, 0, 0, out_bf16, None, 0, None, None, 1.0, out)
                pts.append((K, timeit(f)))
            # least squares t = a + b K
            n = len(pts)
            sk = sum(k for k, _ in pts); st = sum(t for _, t in pts)
            skk = sum(k * k for k, _ in pts); skt = sum(k * t for k, t in pts)
            b = (n * skt - sk * st) / (n * skk - sk * sk)
            a = (st - b * sk) / n
            tiles = ((M + 255) // 256) * ((N + 255) // 256)
            print(json.dumps({"M": M, "N": N, "out": "bf16" if out_bf16 else "fp32", "wide": wide, "tiles": tiles,
                              "us": {k: round(t, 1) for k, t in pts}, "fit_a_us": round(a, 1),
                              "fit_us_per_ktile": round(b * 64, 3)}), flush=True)


if __name__ == "__main__":
    main()
