"""128x128 core vs 256x256 kernels on the ViT-B/16 linear shapes (bf16 and fp8 e4m3), to set the tile
heuristics of gemm_bf16 / gemm_fp8 (csrc/kernels/gemm.hip).  python tools/gemm_tile_probe.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C
T = 25216  # tokens of a B=128 ViT-B/16 step


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
    torch.manual_seed(0)
    shapes = [(T, 2304, 768, "qkv fwd"), (T, 768, 768, "proj fwd"), (T, 3072, 768, "fc1 fwd"), (T, 768, 3072, "fc2 fwd"),
              (T, 768, 2304, "qkv dgrad"), (T, 3072, 768, "fc2 dgrad"), (T, 768, 3072, "fc1 dgrad")]
    for M, N, K, note in shapes:
        A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        res = {"shape": f"{M}x{N}x{K}", "note": note}
        for tile in (128, 256):
            C.set_bf16_tile_mode(tile)
            res[f"bf16_{tile}_us"] = round(timeit(lambda: C.gemm(A, B, M, N, K, K, K, False, False, 1, 0, 0, True, None, 0, None, None, 1.0, out)), 1)
        C.set_bf16_tile_mode(0)
        res["bf16_auto_us"] = round(timeit(lambda: C.gemm(A, B, M, N, K, K, K, False, False, 1, 0, 0, True, None, 0, None, None, 1.0, out)), 1)
        if hasattr(C, "gemm_fp8"):
            Aq = A.to(torch.float8_e4m3fn).view(torch.uint8)
            Bq = B.to(torch.float8_e4m3fn).view(torch.uint8)
            one = torch.ones((), device="cuda")
            for tile in (128, 256):
                C.set_fp8_tile_mode(tile)
                try:
                    res[f"fp8_{tile}_us"] = round(timeit(lambda: C.gemm_fp8(Aq, Bq, one, one, M, N, K, True)), 1)
                except Exception as e:  # noqa: BLE001
                    res[f"fp8_{tile}_us"] = str(e)[:60]
            C.set_fp8_tile_mode(0)
        res["TF_bf16_best"] = round(2 * M * N * K / min(res["bf16_128_us"], res["bf16_256_us"]) / 1e6, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
