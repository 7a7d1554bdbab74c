"""Time the fused attention kernels on the ViT-B/16 B=128 shapes (T=197, H=12, head dim 64).
python tools/attn_bench.py"""
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C


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
    B, T, H, D = 128, 197, 12, 64
    torch.manual_seed(0)
    qkv = (torch.randn(B * T, 3 * H * D, device="cuda") * 0.5).bfloat16()
    scale = D ** -0.5
    p, out = C.attn_fwd_rows(qkv, B, T, H, scale)
    dout = torch.randn_like(out)
    t_f = timeit(lambda: C.attn_fwd_rows(qkv, B, T, H, scale))
    t_b = timeit(lambda: C.attn_bwd_rows(dout, qkv, p, B, T, H, scale))
    fl = 4.0 * B * H * T * T * D
    print(f"attn fwd {t_f:.1f} us ({fl / t_f / 1e6:.0f} TFLOP/s), bwd {t_b:.1f} us ({2.5 * fl / t_b / 1e6:.0f} TFLOP/s), "
          f"P {p.numel() * 2 / 1e6:.0f} MB")


if __name__ == "__main__":
    main()
