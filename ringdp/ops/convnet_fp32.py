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

import os

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
        ctx.set_materialize_grads(False)
        return a, code

    @staticmethod
    def backward(ctx, da, _dcode):
        if da is None:
            return (None,) * 7
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
        ctx.set_materialize_grads(False)
        return a, code

    @staticmethod
    def backward(ctx, da, _dcode):
        if da is None:
            return (None,) * 5
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


# Batches up to RINGDP_F32_NET_NODE_MAX_B (4096; 0 disables): ringdp's cross entropy on these logits is ONE autograd
# node over the whole network (_NetCEF32) whose backward runs every layer's gradient kernels and then a single
# launch for all of their weight-gradient reductions (instead of one or two per layer).  Above it the per-layer
# nodes stay, so DDP can all-reduce the fc1 / conv3 bucket while conv2 / conv1 backward still run.
_NET_NODE_MAX_B = int(os.environ.get("RINGDP_F32_NET_NODE_MAX_B", "4096"))


class _NetCEF32(torch.autograd.Function):
    """Cross entropy on the fp32 ConvNet's logits as one node over every layer (small batches).

    The forward reuses the logits and activations of the per-layer forward.  The backward is the per-layer
    backward's sequence (cross-entropy gradient, fc1, pool3, conv3, pool2, conv2, conv1) with two fusions: the
    cross-entropy backward, fc1's data gradient and pool3's backward are one launch, and the weight-gradient
    reductions of all four layers run as one launch at the end (the same fixed-order sums as the per-layer path).  Deferral is safe by construction: every gradient this node returns
    is written before it returns, and autograd reads a node's gradients only after it returns."""

    @staticmethod
    def forward(ctx, w1, b1, w2, b2, w3, b3, wfc, bfc, logits, target, saved, ignore_index, eps, reduction):
        loss, lse, ws = C.cross_entropy_fwd(logits, target, ignore_index, eps, reduction)
        ctx.save_for_backward(logits, target, lse, ws)
        ctx.saved_acts = saved
        ctx.params = (w1, b1, w2, b2, w3, b3, wfc, bfc)
        ctx.cfg = (ignore_index, eps, reduction)
        return loss

    @staticmethod
    def backward(ctx, grad_out):
        logits, target, lse, ws = ctx.saved_tensors
        x, a1, code1, a2, code2, a3, code3, mean, std = ctx.saved_acts
        w1, b1, w2, b2, w3, b3, wfc, bfc = ctx.params
        B = logits.shape[0]
        grads = [grad_buffer(p) for p in (w1, b1, w2, b2, w3, b3, wfc, bfc)]
        dw1, db1, dw2, db2, dw3, db3, dwfc, dbfc = grads
        # cross-entropy backward + fc1 data gradient + pool3 backward: one launch (the logits gradient dl is also
        # written, for fc1's weight gradient)
        dl, dz3 = C.f32_fc_ce_pool3_bwd(logits, target, lse, ws, grad_out.contiguous(), *ctx.cfg, wfc.detach(), code3)
        segs = []
        # fc1's weight gradient (a 1x1 conv over the flattened 2048-vector)
        dz = dl.view(B, -1, 1, 1)
        x3 = a3.reshape(B, -1, 1, 1)
        segs.append(C.f32_conv_wgrad_slab(dz, x3, 0, 0.0, 1.0, dwfc.view(wfc.shape[0], -1, 1, 1), True) + (dwfc, dbfc))
        # conv3 (its data gradient's split-K planes summed inside pool2's 2x2 / s1 backward)
        segs.append(C.f32_conv_wgrad_slab(dz3, a2, 0, 0.0, 1.0, dw3, True) + (dw3, db3))
        dz2 = C.f32_conv_dgrad_pool2s1_bwd(dz3, w3.detach(), code2)
        # conv2
        da1 = C.f32_conv_dgrad(dz2, w2.detach(), a1.shape[2], a1.shape[3], 0)
        segs.append(C.f32_conv_wgrad_slab(dz2, a1, 0, 0.0, 1.0, dw2, True) + (dw2, db2))
        # conv1 (+ pool1, folded into its weight gradient)
        segs.append(C.f32_conv1_wgrad_slab(x, da1, code1, mean, std) + (dw1, db1))
        C.f32_slab_reduce_multi([sg[0] for sg in segs], [sg[1] for sg in segs], [sg[2] for sg in segs],
                                [sg[3] for sg in segs])
        n = ctx.needs_input_grad
        return tuple(g if need else None for g, need in zip(grads, n[:8])) + (None,) * 6


def head_cross_entropy_fp32(logits: torch.Tensor, target: torch.Tensor, ignore_index: int, eps: float,
                            reduction: int):
    """The whole-network fp32 node when ``logits`` is the untouched output of ``convnet_forward_fp32`` at a small
    batch, else None.  Called by ringdp.ops.loss.cross_entropy."""
    net = getattr(logits, "_ringdp_net32", None)
    if net is None or not torch.is_grad_enabled() or not logits.requires_grad:
        return None
    if target.dim() != 1 or target.shape[0] != logits.shape[0] or not target.is_cuda:
        return None
    params, saved, version, node = net
    if logits._version != version or logits.grad_fn is not node or logits.retains_grad or logits._backward_hooks:
        return None
    if not all(p.requires_grad for p in params):
        return None
    return _NetCEF32.apply(*params, logits.detach(), target.long().contiguous(), saved, ignore_index, eps, reduction)


def convnet_forward_fp32(x: torch.Tensor, conv1, conv2, conv3, fc1) -> torch.Tensor:
    """fp32 GPU forward of the reference ConvNet (ref/launch_dist.py:35-41): uint8 pixels
    (normalised in conv1's loads) or already-normalised float input; fp32 logits [B, 10]."""
    if x.dtype == torch.uint8:
        mean, std = MNIST_MEAN, MNIST_STD
    else:
        x = x.float()
        mean, std = 0.0, 1.0
    x = x.contiguous()
    dedicated1 = x.shape[1:] == (1, 28, 28) and conv1.bias is not None and not x.requires_grad
    if dedicated1:
        a1, code1 = _Conv1PoolF32.apply(x, conv1.weight, conv1.bias, mean, std)
    else:
        a1, code1 = _ConvPoolF32.apply(x, conv1.weight, conv1.bias, 1, mean, std)
    a2, code2 = _ConvPoolF32.apply(a1, conv2.weight, conv2.bias, 0, 0.0, 1.0, 1)
    a3, code3 = _ConvPoolF32.apply(a2, conv3.weight, conv3.bias, 0, 0.0, 1.0)
    logits = _ConvF32.apply(a3.reshape(a3.shape[0], -1), fc1.weight, fc1.bias, 0, 0.0, 1.0)
    if (logits.requires_grad and dedicated1 and x.shape[0] <= _NET_NODE_MAX_B and a3.shape[1:] == (128, 4, 4)
            and all(m.bias is not None for m in (conv2, conv3, fc1))):
        # what ringdp's cross entropy needs to run the whole backward as one node (head_cross_entropy_fp32)
        params = (conv1.weight, conv1.bias, conv2.weight, conv2.bias, conv3.weight, conv3.bias, fc1.weight, fc1.bias)
        saved = (x, a1.detach(), code1, a2.detach(), code2, a3.detach(), code3, mean, std)
        logits._ringdp_net32 = (params, saved, logits._version, logits.grad_fn)
    return logits
