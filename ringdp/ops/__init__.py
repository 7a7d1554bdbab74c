"""ringdp.ops - autograd Functions over ringdp's CDNA4 HIP kernels.

Gradient "slots": when a parameter is managed by ringdp's DDP, its gradient lives in a flat
all-reduce bucket.  Ops write weight gradients straight into that slot (``grad_buffer``) and
autograd's AccumulateGrad adopts the tensor without a copy, so the reducer never runs a
flatten/copy kernel (SURVEY.md §2.6 K23/K24 eliminated).
"""
from __future__ import annotations

import torch

from .._native import C


def grad_buffer(param: torch.Tensor) -> torch.Tensor:
    """A tensor to write ``param``'s gradient into: its DDP bucket slot when the parameter has no
    accumulated gradient yet (AccumulateGrad then adopts it as-is), otherwise fresh memory."""
    slot = getattr(param, "_ringdp_grad_slot", None)
    if slot is not None and param.grad is None and slot.shape == param.shape:
        return slot.detach()  # fresh TensorImpl aliasing the slot (keeps AccumulateGrad's steal path)
    return torch.empty_like(param, memory_format=torch.contiguous_format)


def require_gpu_kernel(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(f"ringdp.ops.{what}: expected a GPU tensor")


from . import convnet, loss  # noqa: E402,F401
