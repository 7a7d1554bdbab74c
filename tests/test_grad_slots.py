"""Grad-as-bucket-view slots (ringdp.ops.grad_buffer) with a parameter that feeds two autograd nodes
in one backward (a slot handed to both nodes summed to 2 x the last partial gradient).
CPU, fake process group: the op below writes its weight gradient through grad_buffer exactly like
the HIP ops do."""
import torch
import torch.nn as nn

import ringdp.distributed as dist
from ringdp.ops import grad_buffer


class _SlotLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x)
        ctx.w = w
        return x @ w.t()

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dw = grad_buffer(ctx.w)
        torch.mm(dy.t(), x, out=dw)
        return dy @ ctx.w, dw


class Twice(nn.Module):
    def __init__(self, slot_op: bool):
        super().__init__()
        self.w = nn.Parameter(torch.randn(8, 8) * 0.3)
        self.slot_op = slot_op

    def forward(self, x):
        f = (lambda a: _SlotLinear.apply(a, self.w)) if self.slot_op else (lambda a: a @ self.w.t())
        return f(torch.tanh(f(x)))  # the same weight used by two nodes


def test_shared_weight_gradient_is_sum_of_both_uses():
    from ringdp.parallel import DistributedDataParallel as DDP

    dist.init_process_group("fake", rank=0, world_size=2)
    try:
        torch.manual_seed(0)
        m = Twice(slot_op=True)
        ref = Twice(slot_op=False)
        ref.load_state_dict(m.state_dict())
        ddp = DDP(m)
        for it in range(3):
            x = torch.randn(4, 8)
            ddp(x).square().sum().backward()
            ref(x).square().sum().backward()
            assert torch.allclose(m.w.grad, ref.w.grad, atol=1e-5, rtol=1e-5), it
            # the gradient still ends up in the bucket slot (grad-as-bucket-view)
            assert m.w.grad.data_ptr() == m.w._ringdp_grad_slot.data_ptr()
            m.w.grad = None
            ref.w.grad = None
    finally:
        dist.destroy_process_group()
