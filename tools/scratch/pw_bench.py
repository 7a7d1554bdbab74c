"""ResNet-50 (B=256) pointwise-conv GEMMs: ringdp's conv2d_fwd (GEMM core + BN-statistics epilogue) and
conv2d_dgrad against torch.matmul (hipBLASLt) and the HBM floor (bytes moved / 5 TB/s).
Usage: python tools/pw_bench.py [B]"""
import json
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C


def timeit(fn, iters=10, warm=3):
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
    return a.elapsed_time(b) / iters * 1000.0


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    shapes = [(56, 64, 256), (56, 256, 64), (56, 64, 64), (28, 128, 512), (28, 512, 128), (14, 256, 1024),
              (14, 1024, 256), (7, 512, 2048), (7, 2048, 512)]
    for hw, cin, cout in shapes:
        M = B * hw * hw
        x = torch.randn(B, hw, hw, cin, device="cuda").bfloat16()
        w = torch.randn(cout, cin, 1, 1, device="cuda") * 0.05
        krsc, crsk = C.pack_conv_weight(w, cin)
        t_fwd = timeit(lambda: C.conv2d_fwd(x, krsc, 1, 0, 1, True))
        t_fwd_ns = timeit(lambda: C.conv2d_fwd(x, krsc, 1, 0, 1, False))
        x2 = x.view(M, cin)
        wt = w.view(cout, cin).bfloat16()
        t_mm = timeit(lambda: torch.matmul(x2, wt.t()))
        dz = torch.randn(B, hw, hw, cout, device="cuda").bfloat16()
        t_dg = timeit(lambda: C.conv2d_dgrad(dz, crsk, hw, hw, 1, 0, 1, None))
        wc = wt.contiguous()
        t_mm_dg = timeit(lambda: torch.matmul(dz.view(M, cout), wc))
        dw = torch.empty(cout, cin, 1, 1, device="cuda")
        t_wg = timeit(lambda: C.conv2d_wgrad(dz, x, dw, 1, 0, 1))
        t_mm_wg = timeit(lambda: torch.matmul(dz.view(M, cout).t(), x2))
        floor = (M * cin + M * cout) * 2 / 5e12 * 1e6
        print(json.dumps({"hw": hw, "cin": cin, "cout": cout, "M": M, "fwd_stats_us": round(t_fwd, 1),
                          "fwd_nostats_us": round(t_fwd_ns, 1), "matmul_us": round(t_mm, 1),
                          "dgrad_us": round(t_dg, 1), "matmul_dgrad_us": round(t_mm_dg, 1),
                          "wgrad_us": round(t_wg, 1), "matmul_wgrad_us": round(t_mm_wg, 1),
                          "hbm_floor_us": round(floor, 1)}), flush=True)


if __name__ == "__main__":
    main()
