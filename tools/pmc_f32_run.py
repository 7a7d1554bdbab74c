"""fp32 ConvNet GEMMs at conv3 / conv2 shape for PMC passes: python tools/pmc_f32_run.py [B] [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ringdp  # noqa: E402

C = ringdp._C
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda")
torch.manual_seed(0)
for cin, h, cout in ((64, 10, 128), (32, 13, 64)):
    x = torch.randn(B, cin, h, h, device=dev)
    w = torch.randn(cout, cin, 3, 3, device=dev) * 0.1
    b = torch.randn(cout, device=dev)
    dw, db = torch.empty_like(w), torch.empty_like(b)
    for _ in range(iters):
        z = C.f32_conv_fwd(x, w, b, 0)
        C.f32_conv_dgrad(z, w, h, h, 0)
        C.f32_conv_wgrad(z, x, 0, 0.0, 1.0, dw, db)
torch.cuda.synchronize()
print("done")
