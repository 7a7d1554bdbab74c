"""Autograd Functions for the MNIST ConvNet hot path (csrc/kernels/convnet.hip).

Forward is three fused blocks (reference layers ref/launch_dist.py:35-41):

* ``_Conv1``  conv1 + ReLU + pool1 (+ fused ToTensor/Normalize for uint8 input) -> a1
* ``_Conv2``  conv2 + bias + ReLU + overlapping pool2 -> a2 and one pool2 code byte per value
* ``_Conv3FC``  conv3 + ReLU + pool3 + view + fc1 -> logits

By default conv1 and conv2 form one node (``_Conv12``) whose backward is a single fused kernel: conv2's
data gradient da1 stays in LDS and feeds conv1's weight gradient directly.

conv2's pre-activation z2 is never materialised.  ``_Conv2`` returns a zero-stride placeholder
for it (autograd's handle on "the gradient of conv2's output") next to the real activations;
``_Conv3FC``'s backward scatters d(a2) through the pool2 codes straight into dz2, so conv2's
backward is a plain linear-layer backward and pool2/ReLU backward costs no extra pass over
memory.  Weights live as bf16 MFMA fragments (``C.cn_pack_weights`` layout) next to the fp32 master
parameters; on the default path ringdp.optim.SGD writes the fragments as it updates the masters
(``PackState``), so the forward packs only when no optimizer step wrote them since the last forward
(``invalidate_pack`` covers raw writes in between).  Autograd fires parameter hooks block by block - fc1/conv3 grads are final after
``_Conv3FC.backward`` - so ringdp's reducer starts the first bucket all-reduce while conv2/conv1
backward kernels still run.
"""
from __future__ import annotations

import os
import weakref

import torch

from .._native import C
from . import grad_buffer

# RINGDP_CN_FUSE12=0: conv1 / conv2 as separate autograd nodes with their own backward kernels (A/B)
_FUSE12 = os.environ.get("RINGDP_CN_FUSE12", "1") != "0"
# RINGDP_CN_FUSED_FWD=0: the three-launch forward (conv1+pack / conv2 / conv3+fc1) instead of the
# whole-forward kernel (weight pack + cn_forward_fused; B=65536: forward 1469 -> 1390 us, B=100: 28 -> 23 us)
_FUSED_FWD = os.environ.get("RINGDP_CN_FUSED_FWD", "1") != "0"
# RINGDP_CN_DEFER_REDUCE=1: the conv3 / fc1 weight-gradient reduction rides in conv12's reduction launch.
# Opt-in: while deferred, the DDP slots of w3/b3/wfc/bfc hold stale values, and nothing in autograd lets
# this node prove that no other producer (an L2 term on the weights, a tied use) makes the engine sum the
# slot before conv12's backward runs.
_DEFER = os.environ.get("RINGDP_CN_DEFER_REDUCE", "0") == "1"
# RINGDP_CN_HEAD_CE=0: ringdp's cross entropy on the ConvNet logits stays a separate node (A/B)
_HEAD_CE = os.environ.get("RINGDP_CN_HEAD_CE", "1") != "0"
# Batches up to RINGDP_CN_NET_NODE_MAX_B (4096; 0 disables): the fused cross entropy is ONE autograd node over
# the whole network (_NetCE), whose backward is conv3 (+fc1 +CE) backward, conv12 backward and a single
# weight-gradient reduction launch.  Above it the head and conv1/conv2 stay separate nodes, so the fc1/conv3
# gradient bucket can be all-reduced while conv2/conv1 backward still run.
_NET_NODE_MAX_B = int(os.environ.get("RINGDP_CN_NET_NODE_MAX_B", "4096"))


def _defer_reduce(params, grads, need_in: bool) -> bool:
    """May the conv3 / fc1 weight-gradient reduction wait for conv12's backward (one reduction
    launch for the whole backward instead of two)?

    Only when nothing reads those gradients before then: every one of them is written straight
    into its DDP bucket slot (AccumulateGrad adopts the slot, no accumulation kernel reads it),
    the slots belong to the bucket that is all-reduced last (the reducer launches buckets in
    order, after conv12's parameters are ready), and conv12's backward follows (the conv3 input
    needs a gradient).  An end-of-backward callback flushes a deferral that nothing consumed
    (e.g. ``torch.autograd.grad`` restricted to the head parameters)."""
    if not (_DEFER and need_in):
        return False
    for p, g in zip(params, grads):
        slot = getattr(p, "_ringdp_grad_slot", None)
        if slot is None or not getattr(p, "_ringdp_last_bucket", False) or g.data_ptr() != slot.data_ptr():
            return False
    dev = grads[0].get_device()
    torch.autograd.Variable._execution_engine.queue_callback(lambda: C.cn_flush_reduce(dev))
    return True

MNIST_MEAN = 0.1307
MNIST_STD = 0.3081


class _Conv1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, packed, mean, std, in_scale):
        a1, idx = C.cn_conv1_fwd(x, packed, b, mean, std, in_scale)
        ctx.save_for_backward(x, idx)
        ctx.params = (w, b)
        ctx.norm = (mean, std, in_scale)
        return a1

    @staticmethod
    def backward(ctx, da1):
        x, idx = ctx.saved_tensors
        w, b = ctx.params
        need_w, need_b = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        if not (need_w or need_b):
            return (None,) * 7
        dw, db = grad_buffer(w), grad_buffer(b)
        C.cn_conv1_wgrad(x, da1.contiguous(), idx, dw, db, *ctx.norm)
        return None, (dw if need_w else None), (db if need_b else None), None, None, None, None


class _Conv2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a1, w, b, packed):
        a2, idx2 = C.cn_conv2_fwd(a1, packed, b)
        z2 = a2.new_empty((1, 1, 1, 1)).expand(a1.shape[0], 11, 11, 64)  # placeholder, never read
        ctx.mark_non_differentiable(a2, idx2)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(a1, packed)
        ctx.params = (w, b)
        return z2, a2, idx2

    @staticmethod
    def backward(ctx, dz2, _da2, _didx2):
        a1, packed = ctx.saved_tensors
        w, b = ctx.params
        C.cn_flush_reduce(a1.get_device())
        dw, db = grad_buffer(w), grad_buffer(b)
        need_in = ctx.needs_input_grad[0]
        da1 = C.cn_conv2_bwd(a1, dz2.contiguous(), packed, need_in, dw, db)
        return (da1 if need_in else None, dw if ctx.needs_input_grad[1] else None,
                db if ctx.needs_input_grad[2] else None, None)


class _Conv12(torch.autograd.Function):
    """conv1 + pool1 and conv2 + pool2 as one autograd node: the backward is one fused kernel
    (conv2 dgrad + wgrad, conv1 wgrad on the LDS-resident da1) and one reduction launch."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w3, wfc, mean, std, in_scale, bufs=None):
        if bufs is not None:
            # fused forward: _Conv3FC's launch (cn_forward_fused) fills these buffers, stream-ordered
            # before any backward kernel reads them
            a1, idx1, a2, idx2, packed = bufs
        else:
            # conv1's launch also packs every layer's bf16 MFMA fragments (w3 / wfc arrive detached:
            # this node only reads them for the packing)
            a1, idx1, packed = C.cn_conv1_fwd_pack(x, w1, w2, w3, wfc, b1, mean, std, in_scale)
            a2, idx2 = C.cn_conv2_fwd(a1, packed, b2)
        z2 = a2.new_empty((1, 1, 1, 1)).expand(a1.shape[0], 11, 11, 64)  # placeholder, never read
        ctx.mark_non_differentiable(a2, idx2, packed)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(x, idx1, a1, packed)
        ctx.params = (w1, b1, w2, b2)
        ctx.norm = (mean, std, in_scale)
        return z2, a2, idx2, packed

    @staticmethod
    def backward(ctx, dz2, _da2, _didx2, _dpacked):
        x, idx1, a1, packed = ctx.saved_tensors
        w1, b1, w2, b2 = ctx.params
        n = ctx.needs_input_grad
        dz2 = dz2.contiguous()
        if n[1] and n[2] and n[3] and n[4]:
            dw1, db1, dw2, db2 = (grad_buffer(t) for t in (w1, b1, w2, b2))
            # also launches a reduction _Conv3FC / _HeadCE deferred into this one
            C.cn_conv12_bwd(x, idx1, a1, dz2, packed, dw2, db2, dw1, db1, *ctx.norm)
            return None, dw1, db1, dw2, db2, None, None, None, None, None, None
        # partially frozen: the separate kernels
        C.cn_flush_reduce(x.get_device())
        need_c1 = n[1] or n[2]
        dw2, db2 = grad_buffer(w2), grad_buffer(b2)
        da1 = C.cn_conv2_bwd(a1, dz2, packed, need_c1, dw2, db2)
        dw1 = db1 = None
        if need_c1:
            dw1, db1 = grad_buffer(w1), grad_buffer(b1)
            C.cn_conv1_wgrad(x, da1, idx1, dw1, db1, *ctx.norm)
        return (None, dw1 if n[1] else None, db1 if n[2] else None, dw2 if n[3] else None,
                db2 if n[4] else None, None, None, None, None, None, None)


class _Conv3FC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z2, a2, idx2, w3, b3, wfc, bfc, packed, fused=None):
        if fused is not None:  # (x, w1, b1, w2, b2, mean, std, in_scale, a1, idx1, do_pack): the whole forward
            x, w1, b1, w2, b2, mean, std, in_scale, a1, idx1, do_pack = fused
            logits, a3, idx3 = C.cn_forward_fused(x, w1, b1, w2, b2, w3, b3, wfc, bfc, mean, std, in_scale,
                                                  a1, idx1, a2, idx2, packed, do_pack)
        else:
            logits, a3, idx3 = C.cn_conv3_fc_fwd(a2, packed, b3, bfc)
        ctx.mark_non_differentiable(a3, idx3)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(a2, idx2, a3, idx3, wfc, packed)
        ctx.params = (w3, b3, wfc, bfc)
        return logits, a3, idx3

    @staticmethod
    def backward(ctx, dlogits, _da3, _didx3):
        a2, idx2, a3, idx3, wfc_saved, packed = ctx.saved_tensors
        w3, b3, wfc, bfc = ctx.params
        n = ctx.needs_input_grad
        if dlogits is None:
            return (None,) * 9
        grads = [grad_buffer(p) for p in (w3, b3, wfc, bfc)]
        need_in = n[0]
        defer = _defer_reduce((w3, b3, wfc, bfc), grads, need_in)
        dz2 = C.cn_conv3_fc_bwd(a2, idx2, a3, idx3, wfc_saved, dlogits.contiguous(), packed, need_in,
                                *grads, defer_reduce=defer)
        dw3, db3, dwfc, dbfc = grads
        return (dz2 if need_in else None, None, None, dw3 if n[3] else None, db3 if n[4] else None,
                dwfc if n[5] else None, dbfc if n[6] else None, None, None)


class _HeadCE(torch.autograd.Function):
    """Cross entropy straight on the ConvNet head: ``loss = CE(fc1(pool3(relu(conv3(a2)))), y)`` as
    one node whose backward forms d(logits) inside the fc1 backward kernel (no ce_bwd launch, no
    [B,10] gradient tensor).  The forward reuses the logits ``_Conv3FC`` already computed; that
    node stays in the graph for any other use of the logits, so gradients through other paths are
    unchanged (the engine sums them)."""

    @staticmethod
    def forward(ctx, z2, w3, b3, wfc, bfc, logits, target, head, ignore_index, eps, reduction):
        loss, lse, ws = C.cross_entropy_fwd(logits, target, ignore_index, eps, reduction)
        ctx.save_for_backward(logits, target, lse, ws)
        ctx.head = head
        ctx.params = (w3, b3, wfc, bfc)
        ctx.cfg = (ignore_index, eps, reduction)
        return loss

    @staticmethod
    def backward(ctx, grad_out):
        logits, target, lse, ws = ctx.saved_tensors
        a2, idx2, a3, idx3, packed = ctx.head
        w3, b3, wfc, bfc = ctx.params
        n = ctx.needs_input_grad
        grads = [grad_buffer(p) for p in (w3, b3, wfc, bfc)]
        need_in = n[0]
        defer = _defer_reduce((w3, b3, wfc, bfc), grads, need_in)
        dz2 = C.cn_conv3_fc_ce_bwd(a2, idx2, a3, idx3, wfc.detach(), logits, target, lse, ws,
                                   grad_out.contiguous(), *ctx.cfg, packed, need_in, *grads, defer)
        dw3, db3, dwfc, dbfc = grads
        return (dz2 if need_in else None, dw3 if n[1] else None, db3 if n[2] else None,
                dwfc if n[3] else None, dbfc if n[4] else None) + (None,) * 6


class _NetCE(torch.autograd.Function):
    """Cross entropy on the ConvNet logits as ONE node over every layer (small batches, see _NET_NODE_MAX_B).

    The forward reuses the logits and activations of the fused forward.  The backward forms d(logits) inside
    the fc1 backward, runs conv3's backward with its weight-gradient reduction deferred, then conv2's backward +
    conv1's weight gradient, whose reduction launch also reduces the deferred conv3 / fc1 slabs: one reduction
    launch per step instead of two.  Deferral is safe by construction here: every gradient slot
    it leaves pending is written before this node returns, and autograd reads a node's gradients only after
    it returns, so another producer of the same weight (a penalty term, a tied use) is summed with the final
    values in stream order."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w3, b3, wfc, bfc, logits, target, saved, ignore_index, eps, reduction):
        loss, lse, ws = C.cross_entropy_fwd(logits, target, ignore_index, eps, reduction)
        ctx.save_for_backward(logits, target, lse, ws)
        ctx.saved_acts = saved
        ctx.params = (w1, b1, w2, b2, w3, b3, wfc, bfc)
        ctx.cfg = (ignore_index, eps, reduction)
        return loss

    @staticmethod
    def backward(ctx, grad_out):
        logits, target, lse, ws = ctx.saved_tensors
        x, idx1, a1, a2, idx2, a3, idx3, packed, norm = ctx.saved_acts
        w1, b1, w2, b2, w3, b3, wfc, bfc = ctx.params
        n = ctx.needs_input_grad
        g3 = [grad_buffer(p) for p in (w3, b3, wfc, bfc)]
        dz2 = C.cn_conv3_fc_ce_bwd(a2, idx2, a3, idx3, wfc.detach(), logits, target, lse, ws,
                                   grad_out.contiguous(), *ctx.cfg, packed, True, *g3, True)
        dw1, db1, dw2, db2 = (grad_buffer(t) for t in (w1, b1, w2, b2))
        # also launches the reduction of the deferred conv3 / fc1 weight-gradient slabs
        C.cn_conv12_bwd(x, idx1, a1, dz2, packed, dw2, db2, dw1, db1, *norm)
        grads = (dw1, db1, dw2, db2) + tuple(g3)
        return (None,) + tuple(g if need else None for g, need in zip(grads, n[1:9])) + (None,) * 6


def head_cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int, eps: float,
                       reduction: int):
    """Fused head + cross entropy when ``logits`` is a ConvNet head output (see ``_HeadCE``), else
    None.  Called by ringdp.ops.loss.cross_entropy."""
    head = getattr(logits, "_ringdp_head", None)
    if head is None or not _HEAD_CE or not torch.is_grad_enabled() or not logits.requires_grad:
        return None
    if target.dim() != 1 or target.shape[0] != logits.shape[0] or not target.is_cuda:
        return None
    z2, a2, idx2, w3, b3, wfc, bfc, packed, a3, idx3, version, node, net = head
    # The fused loss reads logits.detach(): only exact when the logits are still the untouched output of
    # _Conv3FC (an in-place edit bumps the version and replaces grad_fn) and nobody observes their gradient
    # (tensor hooks, retain_grad) - otherwise the plain criterion, whose backward runs through _Conv3FC.
    if logits._version != version or logits.grad_fn is not node or logits.retains_grad \
            or logits._backward_hooks:
        return None
    if net is not None and logits.shape[0] <= _NET_NODE_MAX_B:
        x, idx1, a1, w1, b1, w2, b2, norm = net
        # every weight must want a gradient: partially frozen models keep the per-block nodes
        if all(p.requires_grad for p in (w1, b1, w2, b2, w3, b3, wfc, bfc)):
            return _NetCE.apply(x, w1, b1, w2, b2, w3, b3, wfc, bfc, logits.detach(), target.long().contiguous(),
                                (x, idx1, a1, a2, idx2, a3, idx3, packed, norm), ignore_index, eps, reduction)
    return _HeadCE.apply(z2, w3, b3, wfc, bfc, logits.detach(), target.long().contiguous(),
                         (a2, idx2, a3, idx3, packed), ignore_index, eps, reduction)


class PackState:
    """The ConvNet's packed bf16 MFMA weight fragments, kept across steps.

    ringdp.optim.SGD's flat step writes the fragments of every weight it updates
    (``C.sgd_flat(..., packed=buf)``) and then marks them written (``mark_written``: ``fresh`` plus the
    weights' (version, address) ``key``).  A forward skips packing only when BOTH hold - the fragments were
    written by the optimizer since the last forward, and no version bump happened since - and consumes
    ``fresh``.  So any change of the masters between two forwards without an optimizer step between them
    repacks, including writes that bump no version (``p.data.mul_``, a broadcast into the raw storage).  The
    one window left, an outside write between ``optimizer.step()`` and the next forward that bumps no version,
    is closed by ``invalidate_pack(model)``; ringdp's own raw writers (checkpoint.load, DDP.join) call it.

    Captured steps: a forward captured with the optimizer's fragments never packs at replay, so
    ``StepGraph.replay`` repacks eagerly (``repack``) when a weight's version moved or the state was
    invalidated since the capture (load_state_dict, an EMA copy, ``invalidate_pack``)."""

    __slots__ = ("buf", "key", "fresh", "ws", "__weakref__")

    def __init__(self):
        self.buf = None
        self.key = None
        self.fresh = False
        self.ws = ()

    @staticmethod
    def key_of(ws):
        return tuple((w._version, w.data_ptr()) for w in ws)

    def mark_written(self, ws):
        """The optimizer wrote every fragment from the updated masters."""
        self.key = self.key_of(ws)
        self.fresh = True

    def invalidate(self):
        """The masters changed behind the fragments' back: the next forward (or replay) repacks."""
        self.key = None
        self.fresh = False

    def consume(self, ws) -> bool:
        """Forward: True when it must pack the fragments itself."""
        key = self.key_of(ws)
        do_pack = not (self.fresh and self.key == key)
        self.key, self.fresh = key, False
        return do_pack

    def stale(self) -> bool:
        return self.buf is not None and bool(self.ws) and self.key != self.key_of(self.ws)

    def repack(self):
        """Rebuild the fragments from the masters now (stream-ordered on the current stream)."""
        with torch.no_grad():
            C.cn_pack_weights(*self.ws, out=self.buf)
        self.mark_written(self.ws)


_PACK_STATES: "weakref.WeakSet[PackState]" = weakref.WeakSet()


def pack_states():
    """Every live ConvNet fragment cache (StepGraph checks them before each replay)."""
    return [st for st in list(_PACK_STATES) if st.buf is not None]


def invalidate_pack(model_or_params) -> None:
    """Declare that ConvNet weights were written without a version bump (``p.data`` in-place edits, raw
    broadcasts): the next forward, or the next replay of a captured step, repacks their bf16 fragments.
    Accepts a module (DDP wrappers included) or an iterable of parameters."""
    params = model_or_params.parameters() if hasattr(model_or_params, "parameters") else model_or_params
    for p in params:
        t = getattr(p, "_ringdp_pack", None)
        if t is not None:
            t[0].invalidate()


def _pack_state(conv1, conv2, conv3, fc1):
    st = conv1.__dict__.get("_ringdp_pack_state")
    if st is None:
        st = PackState()
        conv1.__dict__["_ringdp_pack_state"] = st
        _PACK_STATES.add(st)
    ws = (conv1.weight, conv2.weight, conv3.weight, fc1.weight)
    if len(st.ws) != 4 or any(a is not b for a, b in zip(st.ws, ws)):
        st.ws = ws
    for slot, w in enumerate(ws):  # the optimizer finds the fragments through the parameters
        t = getattr(w, "_ringdp_pack", None)
        if t is None or t[0] is not st or t[1] != slot:
            w._ringdp_pack = (st, slot)
    return st, ws


def pack_weights(conv1, conv2, conv3, fc1) -> torch.Tensor:
    with torch.no_grad():
        return C.cn_pack_weights(conv1.weight, conv2.weight, conv3.weight, fc1.weight)


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
    fused = None
    net = None
    if _FUSE12 and _FUSED_FWD:
        st, ws = _pack_state(conv1, conv2, conv3, fc1)
        bufs = C.cn_forward_buffers(x)
        if st.buf is None or st.buf.device != x.device:
            st.buf = bufs[4]
            st.invalidate()
        bufs = (bufs[0], bufs[1], bufs[2], bufs[3], st.buf)
        do_pack = st.consume(ws)  # False: the optimizer wrote these weights' fragments since the last forward
        z2, a2, idx2, packed = _Conv12.apply(x, conv1.weight, conv1.bias, conv2.weight, conv2.bias,
                                             conv3.weight.detach(), fc1.weight.detach(), mean, std, scale, bufs)
        fused = (x, conv1.weight.detach(), conv1.bias.detach(), conv2.weight.detach(), conv2.bias.detach(),
                 mean, std, scale, bufs[0], bufs[1], do_pack)
        net = (x, bufs[1], bufs[0], conv1.weight, conv1.bias, conv2.weight, conv2.bias, (mean, std, scale))
    elif _FUSE12:
        z2, a2, idx2, packed = _Conv12.apply(x, conv1.weight, conv1.bias, conv2.weight, conv2.bias,
                                             conv3.weight.detach(), fc1.weight.detach(), mean, std, scale)
    else:
        packed = pack_weights(conv1, conv2, conv3, fc1)
        a1 = _Conv1.apply(x, conv1.weight, conv1.bias, packed, mean, std, scale)
        z2, a2, idx2 = _Conv2.apply(a1, conv2.weight, conv2.bias, packed)
    logits, a3, idx3 = _Conv3FC.apply(z2, a2, idx2, conv3.weight, conv3.bias, fc1.weight, fc1.bias, packed,
                                      fused)
    if logits.requires_grad:
        # what ringdp's cross entropy needs to fuse itself into the head (head_cross_entropy)
        logits._ringdp_head = (z2, a2, idx2, conv3.weight, conv3.bias, fc1.weight, fc1.bias, packed, a3, idx3,
                               logits._version, logits.grad_fn, net)
    return logits
