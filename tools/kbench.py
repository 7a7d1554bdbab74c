"""Per-kernel timing of the ConvNet hot path (HIP events, median of N), with achieved TFLOP/s.

python tools/kbench.py [B ...]
"""
import json
import sys

import torch

sys.path.insert(0, ".")
import ringdp  # noqa: E402

C = ringdp._C


def timeit(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000)
    ts.sort()
    return ts[len(ts) // 2]


def run(B):
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
    y = torch.randint(0, 10, (B,), device=dev)
    norm = (0.1307, 0.3081, 1 / 255.0)
    pk = C.cn_pack_weights(w1, w2, w3, wf)
    a1, i1 = C.cn_conv1_fwd(x, pk, b1, *norm)
    a2, i2 = C.cn_conv2_fwd(a1, pk, b2)
    logits, a3, i3 = C.cn_conv3_fc_fwd(a2, pk, b3, bfc)
    dl = torch.randn(B, 10, device=dev)
    dz2 = torch.randn(a2.shape[0], 11, 11, 64, device=a2.device).bfloat16()
    da1 = torch.randn_like(a1)
    dw1, db1 = torch.empty_like(w1), torch.empty_like(b1)
    dw2, db2 = torch.empty_like(w2), torch.empty_like(b2)
    dw3, db3 = torch.empty_like(w3), torch.empty_like(b3)
    dwf, dbf = torch.empty_like(wf), torch.empty_like(bfc)
    c1 = 2 * 26 * 26 * 32 * 25
    c2 = 2 * 121 * 64 * 288
    c3 = 2 * 64 * 128 * 576
    F = {"conv1_fwd": c1, "conv2_fwd": c2, "conv3_fc_fwd": c3 + 2 * 2048 * 10,
         "conv3_fc_bwd": 2 * c3 + 2 * 100 * 64 * 1152, "conv3_fc_bwd_w": c3,
         "conv2_bwd": c2 + 2 * 169 * 32 * 576, "conv2_bwd_w": c2, "conv1_wgrad": c1}
    res = {}
    res["pack"] = timeit(lambda: C.cn_pack_weights(w1, w2, w3, wf))
    res["conv1_fwd"] = timeit(lambda: C.cn_conv1_fwd(x, pk, b1, *norm))
    res["conv2_fwd"] = timeit(lambda: C.cn_conv2_fwd(a1, pk, b2))
    res["conv3_fc_fwd"] = timeit(lambda: C.cn_conv3_fc_fwd(a2, pk, b3, bfc))
    res["ce_fwd"] = timeit(lambda: C.cross_entropy_fwd(logits, y, -100, 0.0, 1))
    res["conv3_fc_bwd"] = timeit(lambda: C.cn_conv3_fc_bwd(a2, i2, a3, i3, wf, dl, pk, True, dw3, db3, dwf, dbf))
    res["conv3_fc_bwd_w"] = timeit(lambda: C.cn_conv3_fc_bwd(a2, i2, a3, i3, wf, dl, pk, False, dw3, db3, dwf, dbf))
    res["conv2_bwd"] = timeit(lambda: C.cn_conv2_bwd(a1, dz2, pk, True, dw2, db2))
    res["conv2_bwd_w"] = timeit(lambda: C.cn_conv2_bwd(a1, dz2, pk, False, dw2, db2))
    res["conv1_wgrad"] = timeit(lambda: C.cn_conv1_wgrad(x, da1, i1, dw1, db1, *norm))
    out = {"B": B}
    for k, v in res.items():
        tf = F.get(k, 0) * B / (v * 1e-6) / 1e12 if k in F else None
        out[k] = {"us": round(v, 1), "TFLOPs": round(tf, 1) if tf else None}
    out["total_us"] = round(sum(v for k, v in res.items() if not k.endswith("_w")), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    for b in (sys.argv[1:] or ["100", "1024", "4096", "16384"]):
        run(int(b))
