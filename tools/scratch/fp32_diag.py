# per-parameter gradient error of the fp32 ConvNet vs ATen fp32 at B=2048 (max-abs, relative L2)
import torch
import torch.nn.functional as F
from ringdp.models import ConvNet

DEV = "cuda"
for B in (64, 2048):
    torch.manual_seed(0)
    m32 = ConvNet(precision="fp32").to(DEV)
    ref = ConvNet().to(DEV)
    ref.load_state_dict(m32.state_dict())
    x = torch.randint(0, 256, (B, 1, 28, 28), dtype=torch.uint8, device=DEV)
    y = torch.randint(0, 10, (B,), device=DEV)
    out = m32(x)
    rout = ref.reference_forward(x)
    print(B, "logits maxabs", float((out - rout).abs().max()), "ref max", float(rout.abs().max()))
    F.cross_entropy(out, y).backward()
    F.cross_entropy(rout, y).backward()
    for (n, p), q in zip(m32.named_parameters(), ref.parameters()):
        d = (p.grad - q.grad)
        print(B, n, "maxabs", float(d.abs().max()), "refmax", float(q.grad.abs().max()),
              "relL2", float(d.norm() / q.grad.norm()))
