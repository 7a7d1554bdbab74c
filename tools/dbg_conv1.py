import sys; sys.path.insert(0,'.')
import torch
import ringdp
C = ringdp._C
dev = torch.device('cuda')
B = 1
x = (torch.arange(784, device=dev, dtype=torch.float32) + 1).view(1, 1, 28, 28) / 1000.0
idx = torch.zeros(B, 13, 32, 16, dtype=torch.uint8, device=dev)
idx[..., :13] = 4
for (py, px, co) in [(0, 0, 0), (0, 1, 0), (0, 0, 1), (1, 0, 0), (0, 5, 3), (2, 7, 17), (12, 12, 31)]:
    da1 = torch.zeros(B, 13, 13, 32, device=dev).bfloat16()
    da1[0, py, px, co] = 1.0
    dw = torch.empty(32, 1, 5, 5, device=dev); db = torch.empty(32, device=dev)
    C.cn_conv1_wgrad(x, da1, idx, dw, db, 0.0, 1.0, 1.0)
    nz = db.nonzero().flatten().tolist()
    v = dw[nz[0], 0, 1, 1].item() * 1000 if nz else None  # xpad[oh+1][ow+1] = x[oh][ow]
    print((py, px, co), 'db nz', nz, [round(db[i].item(), 3) for i in nz], 'x@', v, 'expect oh,ow', 2 * py, 2 * px,
          '-> val', (2 * py) * 28 + 2 * px + 1)
