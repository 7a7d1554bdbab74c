"""Time the fp8 quantise(+transpose) pass (delayed scaling) on the ViT-B/16 B=128 shapes."""
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C


def main():
    out = []
    for R, Cc in [(25216, 768), (25216, 2304), (25216, 3072), (768, 768), (3072, 768), (2304, 768)]:
        x = torch.randn(R, Cc, device="cuda").bfloat16()
        hist = torch.zeros(1 + C.fp8_delayed_slots(R, Cc), device="cuda")
        C.fp8_quantize_both_delayed(x, hist, True, None, None)
        for _ in range(3):
            C.fp8_quantize_both_delayed(x, hist, False, None, None)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            C.fp8_quantize_both_delayed(x, hist, False, None, None)
        b.record()
        b.synchronize()
        us = a.elapsed_time(b) / 20 * 1000
        out.append(f"{R}x{Cc}: {us:.1f} us ({R * Cc * 4 / us / 1e6:.2f} TB/s)")
    print("; ".join(out))


if __name__ == "__main__":
    main()
