"""ringdp.ops - autograd Functions over ringdp's CDNA4 HIP kernels.

Gradient "slots": when a parameter is managed by ringdp's DDP, its gradient lives in a flat
all-reduce bucket.  Ops write weight gradients straight into that slot (``grad_buffer``) and
autograd's AccumulateGrad adopts the tensor without a copy, so the reducer never runs a
flatten/copy kernel (SURVEY.md §2.6 K23/K24 eliminated).
"""
from __future__ import annotations

import torch

from .._native import C


_backward_epoch = [0]


def next_backward_epoch() -> None:
    """Called by DDP once per forward that will be followed by a backward: grad slots handed out
    from then on belong to that backward."""
    _backward_epoch[0] += 1


def grad_buffer(param: torch.Tensor) -> torch.Tensor:
    """A tensor to write ``param``'s gradient into: its DDP bucket slot when the parameter has no
    accumulated gradient yet (AccumulateGrad then adopts it as-is), otherwise fresh memory.

    The slot is handed out at most once per backward.  A parameter that feeds several autograd
    nodes (tied weights, a layer applied twice) gets one partial gradient per node; the engine
    sums them in its input buffer before AccumulateGrad runs, so every node but the first must
    write into its own memory - two aliases of the slot would sum to 2 x the last write."""
    slot = getattr(param, "_ringdp_grad_slot", None)
    if slot is not None and param.grad is None and slot.shape == param.shape \
            and getattr(param, "_ringdp_slot_epoch", -1) != _backward_epoch[0]:
        param._ringdp_slot_epoch = _backward_epoch[0]
        return slot.detach()  # fresh TensorImpl aliasing the slot (keeps AccumulateGrad's steal path)
    return torch.empty_like(param, memory_format=torch.contiguous_format)


def require_gpu_kernel(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(f"ringdp.ops.{what}: expected a GPU tensor")


from . import convnet, loss  # noqa: E402,F401
