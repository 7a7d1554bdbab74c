"""Where does the 256x256 bf16 GEMM lose time?  For each shape, time the phased kernel and the older
single-stage-wait kernel on (a) the real operands and (b) operands whose rows all alias one row
(lda = ldb = 0: every load hits on-chip caches), which isolates the pipeline from memory locality.
python tools/gemm_probe.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C

SHAPES = [(25216, 2304, 768, "vit qkv"), (25216, 3072, 768, "vit fc1"), (25216, 768, 3072, "vit fc2"),
          (25216, 768, 768, "vit proj"), (4096, 4096, 4096, "sq4k"), (8192, 8192, 8192, "sq8k")]


def timeit(fn, iters=20, warm=3):
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
    C.set_bf16_tile_mode(256)
    for M, N, K, note in SHAPES:
        A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        res = {"shape": f"{M}x{N}x{K}", "note": note}
        fl = 2 * M * N * K
        for phased in (1, 0):
            C.set_gemm256_phased(phased)
            for resident in (False, True):
                ld = 0 if resident else K
                f = lambda: C.gemm(A, B, M, N, K, ld, ld, False, False, 1, 0, 0, True, None, 0, None, None, 1.0, out)
                us = timeit(f)
                res[f"{'p' if phased else 'o'}{'_res' if resident else ''}_TF"] = round(fl / us / 1e6, 1)
        C.set_gemm256_phased(1)
        res["blaslt_TF"] = round(fl / timeit(lambda: torch.matmul(A, B.t())) / 1e6, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
