"""Run one ConvNet kernel group repeatedly for PMC collection under rocprofv3 --pmc.

python tools/pmc_run.py <op> [B] [iters]   op: fwd_fused | fwd_sep | conv3_fc_bwd | conv12_bwd | conv2_bwd | conv3_fc_fwd | conv2_fwd | conv1_fwd | conv1_wgrad
"""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import ringdp  # noqa: E402

C = ringdp._C


def build_ops(B):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = torch.randint(0, 256, (B, 1, 28, 28), dtype=torch.uint8, device=dev)
    w1 = torch.randn(32, 1, 5, 5, device=dev) * 0.2
    b1 = torch.randn(32, device=dev) * 0.1
    w2 = torch.randn(64, 32, 3, 3, device=dev) * 0.1
    b2 = torch.randn(64, device=dev) * 0.1
    w3 = torch.randn(128, 64, 3, 3, device=dev) * 0.1
    b3 = torch.randn(128, device=dev) * 0.1
    wf = torch.randn(10, 2048, device=dev) * 0.05
    bfc = torch.randn(10, device=dev)
    norm = (0.1307, 0.3081, 1.0 / 255.0)
    pk = C.cn_pack_weights(w1, w2, w3, wf)
    a1, i1 = C.cn_conv1_fwd(x, pk, b1, *norm)
    a2, i2 = C.cn_conv2_fwd(a1, pk, b2)
    logits, a3, i3 = C.cn_conv3_fc_fwd(a2, pk, b3, bfc)
    dl = torch.randn(B, 10, device=dev)
    dz2 = torch.randn(B, 11, 11, 64, device=dev).bfloat16()
    da1 = torch.randn(B, 13, 13, 32, device=dev).bfloat16()
    g3 = [torch.empty_like(t) for t in (w3, b3, wf, bfc)]
    g2 = [torch.empty_like(t) for t in (w2, b2)]
    g1 = [torch.empty_like(t) for t in (w1, b1)]
    bufs = C.cn_forward_buffers(x)
    labels = torch.randint(0, 10, (B,), device=dev)
    loss, lse, cews = C.cross_entropy_fwd(logits, labels, -100, 0.0, 1)
    one = torch.ones((), device=dev)

    def fwd_sep():
        a1_, i1_, pk_ = C.cn_conv1_fwd_pack(x, w1, w2, w3, wf, b1, *norm)
        a2_, i2_ = C.cn_conv2_fwd(a1_, pk_, b2)
        return C.cn_conv3_fc_fwd(a2_, pk_, b3, bfc)

    fns = {
        "fwd_fused": lambda: C.cn_forward_fused(x, w1, b1, w2, b2, w3, b3, wf, bfc, *norm, *bufs),
        "fwd_sep": fwd_sep,
        "conv1_fwd": lambda: C.cn_conv1_fwd(x, pk, b1, *norm),
        "conv2_fwd": lambda: C.cn_conv2_fwd(a1, pk, b2),
        "conv3_fc_fwd": lambda: C.cn_conv3_fc_fwd(a2, pk, b3, bfc),
        "conv3_fc_bwd": lambda: C.cn_conv3_fc_bwd(a2, i2, a3, i3, wf, dl, pk, True, *g3),
        "conv3_fc_ce_bwd": lambda: C.cn_conv3_fc_ce_bwd(a2, i2, a3, i3, wf, logits, labels, lse, cews, one, -100,
                                                        0.0, 1, pk, True, *g3, False),
        "conv3_fc_bwd_w": lambda: C.cn_conv3_fc_bwd(a2, i2, a3, i3, wf, dl, pk, False, *g3),
        "conv2_bwd_w": lambda: C.cn_conv2_bwd(a1, dz2, pk, False, *g2),
        "conv2_bwd": lambda: C.cn_conv2_bwd(a1, dz2, pk, True, *g2),
        "conv1_wgrad": lambda: C.cn_conv1_wgrad(x, da1, i1, *g1, *norm),
        "conv12_bwd": lambda: C.cn_conv12_bwd(x, i1, a1, dz2, pk, *g2, *g1, *norm),
    }
    return fns


def main():
    op = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    fns = build_ops(B)
    for _ in range(iters):
        fns[op]()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
