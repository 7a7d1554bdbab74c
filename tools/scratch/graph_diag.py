"""Bisect hipGraph capture of the ConvNet step: fwd / fwd+loss / +backward / +optimizer."""
import sys
import torch
import ringdp, ringdp.distributed as dist
from ringdp.models import ConvNet
from ringdp.nn import CrossEntropyLoss
from ringdp.optim import SGD
from ringdp.parallel import DistributedDataParallel as DDP

level = sys.argv[1]
use_ddp = len(sys.argv) > 2 and sys.argv[2] == "ddp"
torch.cuda.set_device(0)
dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)
torch.manual_seed(0)
m = ConvNet().cuda()
net = DDP(m, device_ids=[0]) if use_ddp else m
opt = SGD(net.parameters(), lr=0.01)
crit = CrossEntropyLoss()
x, y = ringdp._C.synth_u8_images(64, 28, 28, 10, 0, torch.device("cuda", 0))

def step():
    out = net(x)
    if level == "fwd":
        return out
    loss = crit(out, y)
    if level == "loss":
        return loss
    opt.zero_grad(set_to_none=True)
    loss.backward()
    if level == "bwd":
        return loss
    opt.step()
    return loss

for _ in range(2):
    step()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        step()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
print("capturing", level, use_ddp, flush=True)
with torch.cuda.graph(g, capture_error_mode=sys.argv[3] if len(sys.argv) > 3 else "thread_local"):
    out = step()
print("captured", flush=True)
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
print("OK", level, use_ddp, float(out.float().sum()), flush=True)
