"""Autograd Functions for NHWC bf16 conv nets on ringdp's implicit-GEMM kernels (ResNet family).

Reference layers: torchvision ``resnet18`` as used by ``ref/example_mp.py:50`` /
``ref/example_launch.py:26`` (SURVEY.md §2.2 R2, §2.6 K30+).  The fused unit is
``conv -> BatchNorm (batch statistics) [-> + residual] [-> ReLU]``:

* forward: one implicit-GEMM launch writes the conv output z (bf16) AND the per-channel
  sum / sum-of-squares partials from its epilogue; one elementwise launch applies the normalisation,
  the residual add and the ReLU;
* backward: one reduction launch (ReLU mask, the two channel sums, the residual branch's gradient),
  one apply launch (dz), then the data-gradient GEMM (transposed-conv gather) and the
  weight-gradient GEMM (split-K over output positions, fixed-order reduction that also converts
  KRSC back to the parameter's KCRS layout).

Weights stay fp32 masters in PyTorch layout (state_dict-compatible with torchvision); each forward
packs them once to bf16 KRSC (forward) and CRSK (data gradient).
"""
from __future__ import annotations

import torch

from .._native import C
from . import grad_buffer


def _cpad(c: int) -> int:
    return (c + 7) // 8 * 8


def pack_conv_weights(convs) -> dict:
    """bf16 KRSC/CRSK copies of many conv weights in one launch -> {id(conv): (krsc, crsk)}."""
    convs = list(convs)
    flat = C.pack_conv_weights([c.weight for c in convs], [_cpad(c.in_channels) for c in convs])
    return {id(c): (flat[2 * i], flat[2 * i + 1]) for i, c in enumerate(convs)}


def to_nhwc(x: torch.Tensor) -> torch.Tensor:
    """NCHW fp32/bf16 images -> NHWC bf16 with channels padded to a multiple of 8 (no gradient)."""
    return C.nchw_to_nhwc(x.contiguous(), _cpad(x.shape[1]))


def _cba_forward(x, w, gamma, beta, residual, running_mean, running_var, stride, pad, relu, training, momentum, eps,
                 num_batches_tracked, packed=None):
    """conv -> BN [-> + residual] [-> ReLU] forward; returns y and what the backward needs.  ``packed``:
    (KRSC, CRSK) bf16 weights from a model-wide ``pack_conv_weights`` launch, else packed here."""
    krsc, crsk = packed if packed is not None else C.pack_conv_weight(w, x.shape[-1])
    if training:
        z, sums = C.conv2d_fwd(x, krsc, stride, pad, 1, True)
        y, save = C.bn_fwd_train(z, sums, gamma, beta, running_mean, running_var, eps, momentum, residual, relu,
                                 num_batches_tracked)
    else:
        z, _ = C.conv2d_fwd(x, krsc, stride, pad, 1, False)
        scale = gamma * torch.rsqrt(running_var + eps)
        ss = torch.stack([scale, beta - running_mean * scale]).contiguous()
        y = C.bn_fwd_eval(z, ss, residual, relu)
        save = ss
    return y, (z, y, save, crsk)


def _cba_backward(saved, x, dy, w, gamma, beta, cfg, need_dx: bool, need_dw: bool, dx_residual=None,
                  need_g: bool = False):
    """BN backward, then the data gradient (+ dx_residual, summed in the GEMM epilogue) and the weight
    gradient.  Returns (dx, dw, dgamma, dbeta, g) with g = d(pre-activation) (the residual's gradient), None
    unless ``need_g``: then the BN backward neither stores it nor (BN + ReLU) reads y - the ReLU mask is
    re-derived from z and the forward's scale / shift, bit-identically."""
    z, y, save, crsk = saved
    stride, pad, relu, training = cfg
    if not training:
        raise RuntimeError("ConvBNAct: backward through eval-mode batch norm is not supported")
    dgamma, dbeta = grad_buffer(gamma), grad_buffer(beta)
    dz, g = C.bn_bwd(dy.contiguous(), y, z, save, gamma, relu, dgamma, dbeta, need_g)
    dx = None
    if need_dx:
        res = dx_residual.contiguous() if dx_residual is not None else None
        dx = C.conv2d_dgrad(dz, crsk, x.shape[1], x.shape[2], stride, pad, 1, res)
    dw = None
    if need_dw:
        dw = grad_buffer(w)
        C.conv2d_wgrad(dz, x, dw, stride, pad, 1)
    return dx, dw, dgamma, dbeta, g


class ConvBNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, gamma, beta, residual, running_mean, running_var, stride: int, pad: int, relu: bool,
                training: bool, momentum: float, eps: float, num_batches_tracked=None, packed=None):
        y, saved = _cba_forward(x, w, gamma, beta, residual, running_mean, running_var, stride, pad, relu, training,
                                momentum, eps, num_batches_tracked, packed)
        ctx.save_for_backward(x, *saved)
        ctx.params = (w, gamma, beta)
        ctx.cfg = (stride, pad, relu, training)
        ctx.has_res = residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, *saved = ctx.saved_tensors
        w, gamma, beta = ctx.params
        # with a residual in the forward the ReLU mask needs y (z alone does not give it): the stored-g form
        dx, dw, dgamma, dbeta, g = _cba_backward(saved, x, dy, w, gamma, beta, ctx.cfg, ctx.needs_input_grad[0],
                                                 ctx.needs_input_grad[1], need_g=ctx.has_res)
        dres = g if (ctx.has_res and ctx.needs_input_grad[4]) else None
        return dx, dw, dgamma, dbeta, dres, None, None, None, None, None, None, None, None, None, None


class ConvBNActFork(torch.autograd.Function):
    """A block's first conv+BN(+ReLU) that also hands its input on as the block's identity shortcut:
    ``y, identity = ConvBNActFork.apply(x, ...)``.  The shortcut's gradient then arrives in this
    Function's backward and is summed into the conv's data gradient by the GEMM epilogue, instead of
    autograd adding the two gradients of ``x`` in a separate elementwise pass (BasicBlock/Bottleneck
    without downsample)."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, running_mean, running_var, stride: int, pad: int, relu: bool,
                training: bool, momentum: float, eps: float, num_batches_tracked=None, packed=None):
        y, saved = _cba_forward(x, w, gamma, beta, None, running_mean, running_var, stride, pad, relu, training,
                                momentum, eps, num_batches_tracked, packed)
        ctx.save_for_backward(x, *saved)
        ctx.params = (w, gamma, beta)
        ctx.cfg = (stride, pad, relu, training)
        return y, x  # x returned unmodified: autograd makes it a view whose gradient comes back here

    @staticmethod
    def backward(ctx, dy, dident):
        x, *saved = ctx.saved_tensors
        w, gamma, beta = ctx.params
        if dy is None:
            dx = dident
            dw = dgamma = dbeta = None
        else:
            dx, dw, dgamma, dbeta, _ = _cba_backward(saved, x, dy, w, gamma, beta, ctx.cfg, ctx.needs_input_grad[0],
                                                     ctx.needs_input_grad[1], dx_residual=dident)
            if dx is None:
                dx = dident
        return dx, dw, dgamma, dbeta, None, None, None, None, None, None, None, None, None, None


class ConvBNActPair(torch.autograd.Function):
    """Two conv+BN(+ReLU) branches reading the same input (a downsampling block's first conv and its
    projection shortcut).  Backward: the second branch's data-gradient GEMM adds the first's in its
    epilogue, so the two gradients of the input are never summed by a separate pass."""

    @staticmethod
    def forward(ctx, x, w1, gamma1, beta1, rm1, rv1, nbt1, w2, gamma2, beta2, rm2, rv2, nbt2, cfg1, cfg2,
                training: bool, eps1: float, eps2: float, packed1=None, packed2=None):
        (s1, p1, relu1, mom1), (s2, p2, relu2, mom2) = cfg1, cfg2
        y1, saved1 = _cba_forward(x, w1, gamma1, beta1, None, rm1, rv1, s1, p1, relu1, training, mom1, eps1, nbt1,
                                  packed1)
        y2, saved2 = _cba_forward(x, w2, gamma2, beta2, None, rm2, rv2, s2, p2, relu2, training, mom2, eps2, nbt2,
                                  packed2)
        ctx.save_for_backward(x, *saved1, *saved2)
        ctx.params = (w1, gamma1, beta1, w2, gamma2, beta2)
        ctx.cfg = ((s1, p1, relu1, training), (s2, p2, relu2, training))
        return y1, y2

    @staticmethod
    def backward(ctx, dy1, dy2):
        x, *saved = ctx.saved_tensors
        saved1, saved2 = saved[:4], saved[4:]
        w1, gamma1, beta1, w2, gamma2, beta2 = ctx.params
        need_dx = ctx.needs_input_grad[0]
        r1 = r2 = (None,) * 5
        if dy1 is not None:
            r1 = _cba_backward(saved1, x, dy1, w1, gamma1, beta1, ctx.cfg[0], need_dx, ctx.needs_input_grad[1])
        if dy2 is not None:
            r2 = _cba_backward(saved2, x, dy2, w2, gamma2, beta2, ctx.cfg[1], need_dx, ctx.needs_input_grad[7],
                               dx_residual=r1[0])
        dx = r2[0] if r2[0] is not None else r1[0]
        return (dx, r1[1], r1[2], r1[3], None, None, None, r2[1], r2[2], r2[3], None, None, None, None, None, None,
                None, None, None, None)


class MaxPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k: int, stride: int, pad: int):
        y, arg = C.maxpool2d_fwd(x, k, stride, pad)
        ctx.save_for_backward(arg)
        ctx.cfg = (x.shape[1], x.shape[2], k, stride, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        H, W, k, s, p = ctx.cfg
        return C.maxpool2d_bwd(dy.contiguous(), arg, H, W, k, s, p), None, None, None


def _pad_rows(t: torch.Tensor, rows: int) -> torch.Tensor:
    if t.shape[0] == rows:
        return t.contiguous()
    out = torch.zeros((rows,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    out[: t.shape[0]] = t
    return out


class _Head(torch.autograd.Function):
    """Global average pool + fc at few classes (``C.head_ok``): one launch each way (nn.hip head_*_kernel).
    Returns (logits, pooled); pooled (fp32) is what a fused cross entropy's backward needs."""

    @staticmethod
    def forward(ctx, x, w, b):
        logits, pooled = C.head_fwd(x, w.detach(), b.detach())
        ctx.mark_non_differentiable(pooled)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(pooled, w, b)
        ctx.hw = (x.shape[1], x.shape[2])
        return logits, pooled

    @staticmethod
    def backward(ctx, dl, _dpooled):
        if dl is None:
            return None, None, None
        pooled, w, b = ctx.saved_tensors
        dw, db = grad_buffer(w), grad_buffer(b)
        dx = C.head_bwd(dl.float().contiguous(), None, None, None, None, None, -100, 0.0, 1, pooled, w.detach(),
                        *ctx.hw, dw, db)
        n = ctx.needs_input_grad
        return dx if n[0] else None, dw if n[1] else None, db if n[2] else None


class _HeadCE(torch.autograd.Function):
    """Cross entropy straight on the head (``loss = CE(fc(avgpool(x)), y)``) as one node: the backward forms
    d(logits) inside the head's backward kernel (no ce_bwd launch, no [N, J] gradient tensor).  The forward
    reuses the logits ``_Head`` computed; that node stays in the graph for any other use of the logits."""

    @staticmethod
    def forward(ctx, x, w, b, logits, target, pooled, ignore_index, eps, reduction):
        loss, lse, ws = C.cross_entropy_fwd(logits, target, ignore_index, eps, reduction)
        ctx.save_for_backward(logits, target, lse, ws, pooled, w, b)
        ctx.cfg = (ignore_index, eps, reduction)
        ctx.hw = (x.shape[1], x.shape[2])
        return loss

    @staticmethod
    def backward(ctx, grad_out):
        logits, target, lse, ws, pooled, w, b = ctx.saved_tensors
        dw, db = grad_buffer(w), grad_buffer(b)
        dx = C.head_bwd(None, logits, target, lse, ws, grad_out.contiguous(), *ctx.cfg, pooled, w.detach(), *ctx.hw,
                        dw, db)
        n = ctx.needs_input_grad
        return (dx if n[0] else None, dw if n[1] else None, db if n[2] else None) + (None,) * 6


def classifier_head(x: torch.Tensor, fc) -> torch.Tensor:
    """avgpool + fc of NHWC bf16 ``x`` -> fp32 logits: the one-launch head at few classes, else the GEMM path."""
    if fc.bias is not None and C.head_ok(x.shape[-1], fc.out_features):
        logits, pooled = _Head.apply(x, fc.weight, fc.bias)
        if logits.requires_grad:
            # what ringdp's cross entropy needs to fuse itself into the head (head_cross_entropy)
            logits._ringdp_rhead = (x, fc.weight, fc.bias, pooled, logits._version, logits.grad_fn)
        return logits
    return AvgPoolLinear.apply(x, fc.weight, fc.bias)


def head_cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int, eps: float,
                       reduction: int):
    """The fused head + cross entropy node when ``logits`` is the untouched output of ``classifier_head``'s
    one-launch head, else None.  Called by ringdp.ops.loss.cross_entropy."""
    head = getattr(logits, "_ringdp_rhead", None)
    if head is None or not torch.is_grad_enabled() or not logits.requires_grad:
        return None
    if target.dim() != 1 or target.shape[0] != logits.shape[0] or not target.is_cuda:
        return None
    x, w, b, pooled, version, node = head
    if logits._version != version or logits.grad_fn is not node or logits.retains_grad or logits._backward_hooks:
        return None
    return _HeadCE.apply(x, w, b, logits.detach(), target.long().contiguous(), pooled, ignore_index, eps, reduction)


class AvgPoolLinear(torch.autograd.Function):
    """Global average pool (NHWC bf16) + fully connected head -> fp32 logits."""

    @staticmethod
    def forward(ctx, x, w, b):
        n, h, wd, c = x.shape
        pooled = C.avgpool_fwd(x)  # [N, C] bf16
        ncls = w.shape[0]
        npad = _cpad(ncls)
        wb = _pad_rows(w.detach().to(torch.bfloat16), npad)
        logits = C.gemm(pooled, wb, n, npad, c, c, c, False, False, 1, 0, 0, False, _pad_rows(b.detach(), npad))
        ctx.save_for_backward(pooled, wb)
        ctx.params = (w, b)
        ctx.cfg = (h, wd, ncls, npad)
        logits = logits.view(n, npad)
        return logits if npad == ncls else logits[:, :ncls].contiguous()

    @staticmethod
    def backward(ctx, dl):
        pooled, wb = ctx.saved_tensors
        w, b = ctx.params
        h, wd, ncls, npad = ctx.cfg
        n, c = pooled.shape
        n8 = _cpad(n)  # the weight-gradient GEMM reduces over the batch: K % 8 == 0
        dlp = torch.zeros(n8, npad, device=dl.device, dtype=torch.bfloat16)
        dlp[:n, :ncls] = dl
        # d(pooled)[n][c] = sum_j dl[n][j] W[j][c]:  A = dl (K-contig over classes), B = W^T (row-contig)
        dpooled = C.gemm(dlp, wb, n, c, npad, npad, c, False, True, 1, 0, 0, True)
        dx = C.avgpool_bwd(dpooled.view(n, c), h, wd)
        dw = db = None
        if ctx.needs_input_grad[1]:
            # dW[j][c] = sum_n dl[n][j] pooled[n][c]:  A = dl^T (row-contig), B = pooled^T (row-contig)
            full = torch.empty(npad, c, device=dl.device, dtype=torch.float32)
            C.gemm_splitk_f32(dlp, _pad_rows(pooled, n8), npad, c, n8, npad, c, True, True, max(1, n8 // 256), full)
            dw = grad_buffer(w)
            dw.copy_(full[:ncls])
        if ctx.needs_input_grad[2]:
            db = grad_buffer(b)
            db.copy_(dl.float().sum(0))
        return dx, dw, db
