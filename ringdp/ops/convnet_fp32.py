"""The MNIST ConvNet at the reference's fp32 precision (ref/launch_dist.py:50-59).

Layer-by-layer autograd Functions over the exact-f32 MFMA kernels of csrc/kernels/conv_f32.hip:
conv (implicit GEMM; fc1 runs as a 1x1 conv over the flattened 2048-vector), and ReLU fused into
max-pool with a 1-byte argmax code (backward is a gather, deterministic also for the overlapping
2x2/s1 pool2).  Every conv runs ReLU + its pool inside the conv launch (conv1: a dedicated one-wave-
per-image kernel; conv2: one image per tile, pooled from LDS; conv3: window-major output pixels), so
no pre-activation reaches memory.  ToTensor+Normalize of uint8 pixels is fused into conv1's operand loads.  Weight and
bias gradients come out of one split-K GEMM (bias = an extra column of ones) and land directly in
the DDP bucket slots (``grad_buffer``).  ``ConvNet(precision="bf16")`` (ringdp/ops/convnet.py) is
the fused bf16 fast path; this module is what ``ConvNet(precision="fp32")`` and
``bench.py --dtype fp32`` run.
"""
from __future__ import annotations

import torch

from .._native import C
from . import grad_buffer
from .convnet import MNIST_MEAN, MNIST_STD


class _ConvF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, pad, mean, std):
        w4 = w if w.dim() == 4 else w.view(w.shape[0], -1, 1, 1)  # a Linear weight as a 1x1 conv
        if w.dim() != 4:
            x = x.reshape(x.shape[0], -1, 1, 1)
        z = C.f32_conv_fwd(x, w4, b, pad, mean, std)
        ctx.save_for_backward(x)
        ctx.params = (w, b)
        ctx.cfg = (pad, mean, std, w4.shape)
        return z if w.dim() == 4 else z.view(z.shape[0], -1)

    @staticmethod
    def backward(ctx, dz):
        (x,) = ctx.saved_tensors
        w, b = ctx.params
        pad, mean, std, w4shape = ctx.cfg
        dz = dz.contiguous()
        if dz.dim() == 2:
            dz = dz.view(dz.shape[0], -1, 1, 1)
        w4 = w.view(w4shape)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = C.f32_conv_dgrad(dz, w4, x.shape[2], x.shape[3], pad)
            if w.dim() != 4:
                dx = dx.view(dx.shape[0], -1)
        dw = grad_buffer(w)
        db = grad_buffer(b) if b is not None else None
        C.f32_conv_wgrad(dz, x, pad, mean, std, dw.view(w4shape), db)
        return (dx, dw if ctx.needs_input_grad[1] else None,
                db if (b is not None and ctx.needs_input_grad[2]) else None, None, None, None)


class _ConvPoolF32(torch.autograd.Function):
    """conv + bias + ReLU + 2x2/s2 max-pool: one fused forward launch (the conv output is never
    written); backward = the pool gather into dz, then the conv's data / weight gradients."""

    @staticmethod
    def forward(ctx, x, w, b, pad, mean, std, stride=2):
        a, code = C.f32_conv_pool_fwd(x, w, b, pad, mean, std, stride)
        ctx.save_for_backward(x, code)
        ctx.params = (w, b)
        ctx.cfg = (pad, mean, std, stride)
        ctx.mark_non_differentiable(code)
        return a

    @staticmethod
    def backward(ctx, da):
        x, code = ctx.saved_tensors
        w, b = ctx.params
        pad, mean, std, stride = ctx.cfg
        OH, OW = stride * (code.shape[2] - 1) + 2, stride * (code.shape[3] - 1) + 2
        dz = C.f32_pool_relu_bwd(da.contiguous(), code, OH, OW, 2, stride)
        dx = C.f32_conv_dgrad(dz, w, x.shape[2], x.shape[3], pad) if ctx.needs_input_grad[0] else None
        dw = grad_buffer(w)
        db = grad_buffer(b) if b is not None else None
        C.f32_conv_wgrad(dz, x, pad, mean, std, dw, db)
        return (dx, dw if ctx.needs_input_grad[1] else None,
                db if (b is not None and ctx.needs_input_grad[2]) else None, None, None, None, None)


class _Conv1PoolF32(torch.autograd.Function):
    """The ConvNet's conv1 + ReLU + pool1 (csrc/kernels/conv1_f32.hip): one wave per image from an LDS
    copy; backward = the weight / bias gradient straight from the pooled gradient and the code (the
    input needs no gradient)."""

    @staticmethod
    def forward(ctx, x, w, b, mean, std):
        a, code = C.f32_conv1_pool_fwd(x, w, b, mean, std)
        ctx.save_for_backward(x, code)
        ctx.params = (w, b)
        ctx.cfg = (mean, std)
        ctx.mark_non_differentiable(code)
        return a

    @staticmethod
    def backward(ctx, da):
        x, code = ctx.saved_tensors
        w, b = ctx.params
        mean, std = ctx.cfg
        dw, db = grad_buffer(w), grad_buffer(b)
        C.f32_conv1_wgrad(x, da.contiguous(), code, mean, std, dw, db)
        return None, dw, db, None, None


class _PoolReLUF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, k, stride):
        a, code = C.f32_pool_relu_fwd(z, k, stride)
        ctx.save_for_backward(code)
        ctx.cfg = (z.shape[2], z.shape[3], k, stride)
        return a

    @staticmethod
    def backward(ctx, da):
        (code,) = ctx.saved_tensors
        H, W, k, st = ctx.cfg
        return C.f32_pool_relu_bwd(da.contiguous(), code, H, W, k, st), None, None


def convnet_forward_fp32(x: torch.Tensor, conv1, conv2, conv3, fc1) -> torch.Tensor:
    """fp32 GPU forward of the reference ConvNet (ref/launch_dist.py:35-41): uint8 pixels
    (normalised in conv1's loads) or already-normalised float input; fp32 logits [B, 10]."""
    if x.dtype == torch.uint8:
        mean, std = MNIST_MEAN, MNIST_STD
    else:
        x = x.float()
        mean, std = 0.0, 1.0
    x = x.contiguous()
    if x.shape[1:] == (1, 28, 28) and conv1.bias is not None and not x.requires_grad:
        a = _Conv1PoolF32.apply(x, conv1.weight, conv1.bias, mean, std)
    else:
        a = _ConvPoolF32.apply(x, conv1.weight, conv1.bias, 1, mean, std)
    a = _ConvPoolF32.apply(a, conv2.weight, conv2.bias, 0, 0.0, 1.0, 1)
    a = _ConvPoolF32.apply(a, conv3.weight, conv3.bias, 0, 0.0, 1.0)
    return _ConvF32.apply(a.reshape(a.shape[0], -1), fc1.weight, fc1.bias, 0, 0.0, 1.0)
