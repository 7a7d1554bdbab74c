"""Autograd Functions for the MNIST ConvNet hot path (csrc/kernels/convnet.hip).

Layer boundaries are chosen so autograd fires parameter hooks as early as possible: fc1's
gradients are final after ``_FC.backward``, conv3's after ``_ConvReluPool(3).backward``, etc.,
which is what lets ringdp's reducer start the first bucket all-reduce while conv2/conv1
backward kernels are still running.

Activations are NHWC bf16 pooled outputs; weights are fp32 masters (PyTorch layouts).
"""
from __future__ import annotations

import torch

from .._native import C
from . import grad_buffer

MNIST_MEAN = 0.1307
MNIST_STD = 0.3081


class _Conv1ReluPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, mean, std, in_scale):
        a1, idx = C.convnet_conv1_fwd(x, w, b, mean, std, in_scale)
        ctx.save_for_backward(x, a1, idx)
        ctx.params = (w, b)
        ctx.norm = (mean, std, in_scale)
        return a1

    @staticmethod
    def backward(ctx, da1):
        x, a1, idx = ctx.saved_tensors
        w, b = ctx.params
        need_w, need_b = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        if not (need_w or need_b):
            return None, None, None, None, None, None
        dw, db = grad_buffer(w), grad_buffer(b)
        C.convnet_conv1_wgrad(x, da1.contiguous(), idx, a1, dw, db, *ctx.norm)
        return None, (dw if need_w else None), (db if need_b else None), None, None, None


class _ConvReluPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, layer, inp, w, b):
        out, idx = C.convnet_conv_fwd(layer, inp, w, b)
        ctx.save_for_backward(inp, w, out, idx)
        ctx.params = (w, b)
        ctx.layer = layer
        return out

    @staticmethod
    def backward(ctx, dout):
        inp, w_saved, out, idx = ctx.saved_tensors
        w, b = ctx.params
        dw, db = grad_buffer(w), grad_buffer(b)
        need_in = ctx.needs_input_grad[1]
        din = C.convnet_conv_bwd(ctx.layer, inp, w_saved, dout.contiguous(), idx, out, need_in, dw, db)
        return (None, din if need_in else None, dw if ctx.needs_input_grad[2] else None,
                db if ctx.needs_input_grad[3] else None)


class _FC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a3, w, b):
        logits = C.convnet_fc_fwd(a3, w, b)
        ctx.save_for_backward(a3, w)
        ctx.params = (w, b)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        a3, w_saved = ctx.saved_tensors
        w, b = ctx.params
        dw, db = grad_buffer(w), grad_buffer(b)
        da3 = C.convnet_fc_bwd(a3, w_saved, dlogits.contiguous(), dw, db)
        return (da3 if ctx.needs_input_grad[0] else None, dw if ctx.needs_input_grad[1] else None,
                db if ctx.needs_input_grad[2] else None)


def convnet_forward(x: torch.Tensor, conv1, conv2, conv3, fc1) -> torch.Tensor:
    """Fused GPU forward of the reference ConvNet (ref/launch_dist.py:35-41).

    ``x``: [B, 1, 28, 28] uint8 (raw pixels: ToTensor+Normalize fused into conv1) or float32
    (already normalised).  Returns fp32 logits [B, 10]."""
    if x.dtype == torch.uint8:
        mean, std, scale = MNIST_MEAN, MNIST_STD, 1.0 / 255.0
    else:
        x = x.float()
        mean, std, scale = 0.0, 1.0, 1.0
    x = x.contiguous()
    a1 = _Conv1ReluPool.apply(x, conv1.weight, conv1.bias, mean, std, scale)
    a2 = _ConvReluPool.apply(2, a1, conv2.weight, conv2.bias)
    a3 = _ConvReluPool.apply(3, a2, conv3.weight, conv3.bias)
    return _FC.apply(a3, fc1.weight, fc1.bias)
