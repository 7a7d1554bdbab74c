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


def test_last_bucket_marks_follow_the_bucket_layout():
    """DDP marks the parameters of the bucket it all-reduces last (`_ringdp_last_bucket`): the ConvNet ops
    may defer those parameters' final gradient reduction into a later op of the same backward
    (ringdp/ops/convnet.py _defer_reduce).  One bucket: every parameter; small buckets: only the last
    bucket's, re-marked after the rebuild that follows the gradient-ready order."""
    from ringdp.parallel import DistributedDataParallel as DDP

    dist.init_process_group("fake", rank=0, world_size=2)
    try:
        torch.manual_seed(0)
        m = nn.Sequential(nn.Linear(64, 64), nn.Tanh(), nn.Linear(64, 64), nn.Tanh(), nn.Linear(64, 10))
        ddp = DDP(m)
        assert all(p._ringdp_last_bucket for p in m.parameters())
        m2 = nn.Sequential(nn.Linear(64, 64), nn.Tanh(), nn.Linear(64, 64), nn.Tanh(), nn.Linear(64, 10))
        ddp2 = DDP(m2, bucket_cap_mb=0.01, first_bucket_mb=0.01)
        for _ in range(3):  # the rebuild happens after the first iteration
            ddp2(torch.randn(4, 64)).sum().backward()
            for p in m2.parameters():
                p.grad = None
        buckets = [list(b) for b in ddp2.reducer.bucket_indices()]
        assert len(buckets) > 1
        params = list(m2.parameters())
        last = set(buckets[-1])
        for i, p in enumerate(params):
            assert p._ringdp_last_bucket == (i in last), i
        # autograd readies the output layer first: after the rebuild it sits in the first bucket
        assert not params[-1]._ringdp_last_bucket
        del ddp, ddp2
    finally:
        dist.destroy_process_group()
