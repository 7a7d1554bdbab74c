"""Two-workgroups-per-CU 256x128 bf16 GEMM (gemm_bf16_256n_kernel) vs the one-workgroup 256x256 phased kernel
on the ViT-B/16 linear shapes (B=128: 25216 tokens) and a few ResNet-50 pointwise shapes; each case also
checks the 2-WG result against an fp32 matmul of the same bf16 operands.  python tools/gemm_2wg_probe.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C
T = 25216


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


def main():
    torch.manual_seed(0)
    shapes = [(T, 2304, 768, "qkv fwd"), (T, 768, 768, "proj fwd"), (T, 3072, 768, "fc1 fwd"), (T, 768, 3072, "fc2 fwd"),
              (T, 768, 2304, "qkv dgrad"), (T, 3072, 768, "fc2 dgrad"), (T, 768, 3072, "fc1 dgrad"),
              (802816, 256, 64, "r50 s1 expand"), (200704, 512, 128, "r50 s2 expand"), (50176, 1024, 256, "r50 s3 expand"),
              (12544, 2048, 512, "r50 s4 expand"), (8192, 8192, 8192, "square")]
    C.set_bf16_tile_mode(256)
    for M, N, K, note in shapes:
        A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        f = lambda: C.gemm(A, B, M, N, K, K, K, False, False, 1, 0, 0, True, None, 0, None, None, 1.0, out)
        res = {"shape": f"{M}x{N}x{K}", "note": note}
        C.set_gemm_two_wg(0)
        res["us_1wg"] = round(timeit(f), 1)
        for g in (4, 8, 16):
            C.set_gemm_two_wg(1, g)
            res[f"us_2wg_g{g}"] = round(timeit(f), 1)
        res["us_2wg"] = min(res[f"us_2wg_g{g}"] for g in (4, 8, 16))
        C.set_gemm_two_wg(1, 4)
        f()
        ref = (A[:4096].float() @ B.float().t())
        res["max_err_2wg"] = float((out[:4096].float() - ref).abs().max())
        res["ref_absmax"] = float(ref.abs().max())
        fl = 2 * M * N * K
        res["TF_1wg"] = round(fl / res["us_1wg"] / 1e6, 1)
        res["TF_2wg"] = round(fl / res["us_2wg"] / 1e6, 1)
        print(json.dumps(res), flush=True)
    C.set_gemm_two_wg(2)


if __name__ == "__main__":
    main()
