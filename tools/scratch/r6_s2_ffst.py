"""Fused-forward phase stamps (vtmp/ffst.so built with -DRINGDP_FF_STAMPS): three forwards at B=65536."""
import torch
import ringdp
from ringdp.models import ConvNet

torch.cuda.set_device(0)
m = ConvNet().cuda()
x, y = ringdp._C.synth_u8_images(65536, 28, 28, 10, 0, torch.device("cuda", 0))
for _ in range(3):
    out = m(x)
    torch.cuda.synchronize()
print("done", float(out.float().abs().mean()))
