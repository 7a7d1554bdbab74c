"""Reference only (never on ringdp's path): what kernel geometry the vendor library picks for the ViT fc1
shape - run under rocprofv3 --kernel-trace to read its workgroup size, grid, LDS and register counts.
python tools/blaslt_shape_probe.py"""
import torch

A = (torch.rand(25216, 768, device="cuda") * 2 - 1).bfloat16()
B = (torch.rand(3072, 768, device="cuda") * 2 - 1).bfloat16()
for _ in range(5):
    C = A @ B.t()
torch.cuda.synchronize()
