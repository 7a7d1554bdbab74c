"""Where the 256x256 GEMM's per-tile fixed cost goes, on ViT shapes (M=25216): compute-only (store mode 3)
vs real stores, per output-store cache flavour (0 plain, 1 nt, 2 sc1) and kernel (persistent / one
workgroup per tile).  python tools/gemm_epi_probe.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C


def timeit(fn, iters=20, warm=5):
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
    C.set_bf16_tile_mode(256)
    torch.manual_seed(0)
    for M, N, K in ((25216, 3072, 768), (25216, 2304, 768), (25216, 768, 3072), (8192, 8192, 8192)):
        A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        bias = torch.rand(N, device="cuda")
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        pre = torch.empty_like(out)
        res = {"M": M, "N": N, "K": K}
        plain = lambda: C.gemm(A, B, M, N, K, K, K, False, False, 1, 0, 0, True, None, 0, None, None, 1.0, out)
        gelu = lambda: C.gemm(A, B, M, N, K, K, K, False, False, 1, 0, 0, True, bias, 2, None, pre, 1.0, out)
        C.set_gemm256_persist(0)
        C.set_gemm_wide_store(3)
        res["compute_only"] = round(timeit(plain), 1)
        C.set_gemm_wide_store(4)
        res["epilogue_to_sink"] = round(timeit(plain), 1)
        if K == 768 and N == 3072:
            res["gelu_to_sink"] = round(timeit(gelu), 1)
        C.set_gemm_wide_store(2)
        for persist in (0,):
            C.set_gemm256_persist(persist)
            for fl in (0,):
                C.set_gemm_store_cache(fl)
                res[f"p{persist}_c{fl}"] = round(timeit(plain), 1)
                if K == 768 and N == 3072:
                    res[f"p{persist}_c{fl}_gelu"] = round(timeit(gelu), 1)
        C.set_gemm_store_cache(0)
        C.set_gemm256_persist(0)
        res["TF_best"] = round(2 * M * N * K / min(v for k, v in res.items() if k.startswith("p") and "gelu" not in k) / 1e6, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
