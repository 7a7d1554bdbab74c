"""Autograd Functions for transformer blocks (ViT-B/16, BASELINE.json config 5) on ringdp kernels.

Token activations are row-major bf16 ``[rows, D]``.  Every matmul - the linear layers and all six
attention products - is the generic MFMA GEMM core (``csrc/kernels/gemm.hip``) with its fused
epilogue (bias, GELU with the pre-activation kept for backward, residual add); weight gradients use
its split-K fp32 mode straight into the parameter's gradient slot; LayerNorm, softmax, GELU backward
and the head/token layout moves are the row kernels of ``csrc/kernels/vit.hip``.
"""
from __future__ import annotations

import math
import os
import weakref
from typing import Dict, Optional, Tuple

import torch

from .._native import C
from . import grad_buffer

# RINGDP_ATTN_UNFUSED=1: attention forward as two GEMMs + a softmax pass (the path the fused kernel replaced)
_ATTN_UNFUSED = os.environ.get("RINGDP_ATTN_UNFUSED", "0") == "1"
_ATTN_BWD_GEMMS = os.environ.get("RINGDP_ATTN_BWD_GEMMS", "0") == "1"  # dS kernel + batched GEMMs (A/B runs)
# fused attention saves the per-query log-sum-exp and the backward recomputes P (RINGDP_ATTN_RECOMPUTE=0: store P)
_ATTN_RECOMPUTE = os.environ.get("RINGDP_ATTN_RECOMPUTE", "1") == "1"
# LayerNorm backward also emits the column sums of dx (the producing linear's bias gradient)
_LN_COLSUM = os.environ.get("RINGDP_LN_COLSUM", "0") == "1"
_FP8 = {"on": False}


def set_fp8(on: bool = True) -> None:
    """Run the linear layers' forward, data-gradient and weight-gradient GEMMs in e4m3 on the
    block-scaled MFMA (per-tensor current scaling; attention products stay bf16)."""
    _FP8["on"] = bool(on)


def fp8_enabled() -> bool:
    return _FP8["on"]


# {id(weight): bf16 copy} for the forward in progress (VisionTransformer.forward_rows casts every linear
# weight in one launch); empty outside it
_BF16_WEIGHTS: dict = {}


_BF16_WEIGHTS_T: dict = {}  # {id(bf16 copy): its transpose}, for the data-gradient GEMMs

# data-gradient GEMMs on W^T (K-contiguous, the phased 256x256 kernel) instead of row-contiguous W
_DGRAD_WT = os.environ.get("RINGDP_DGRAD_WT", "1") == "1"


def cast_weights(ws) -> None:
    """Cast many fp32 [out, in] weights to bf16 AND bf16 transposed in one launch for the forward in
    progress (see _bf16 / _bf16_t): the backward's data-gradient GEMMs take W^T K-contiguous."""
    ws = [w for w in ws if w.is_cuda and w.dtype == torch.float32 and w.dim() == 2]
    _BF16_WEIGHTS_T.clear()  # the previous step's backward has taken what it needed
    if ws and _FP8["on"]:
        if _FP8_WQ_BATCH and _FP8_DELAYED and _fp8_weights_batched(ws):
            return
        # fp8 linears quantise W / W^T themselves: plain casts only
        for w, b in zip(ws, C.cast_bf16_multi([w.detach().contiguous() for w in ws])):
            _BF16_WEIGHTS[id(w)] = b
        return
    if ws:
        flat = C.cast_bf16_t_multi([w.detach().contiguous() for w in ws])
        for i, w in enumerate(ws):
            _BF16_WEIGHTS[id(w)] = flat[2 * i]
            # keyed by the bf16 copy, which the entry keeps alive (its id cannot be reused meanwhile)
            _BF16_WEIGHTS_T[id(flat[2 * i])] = (flat[2 * i], flat[2 * i + 1])


def clear_weights() -> None:
    _BF16_WEIGHTS.clear()
    _FP8_WEIGHTS.clear()


# fp8: every linear weight's e4m3 copies (q, q^T, scale) from one launch per forward (cast_weights), instead of a
# bf16 cast launch plus one quantisation launch per weight (RINGDP_FP8_WQ_BATCH=0: per weight)
_FP8_WQ_BATCH = os.environ.get("RINGDP_FP8_WQ_BATCH", "1") == "1"
_FP8_WEIGHTS: dict = {}  # {id(weight): (weight, (q, qt, scale))} for the forward in progress


def _fp8_weights_batched(ws) -> bool:
    """Quantise all of ``ws`` (slot 2 delayed-scaling sites) in one launch; False (nothing done) while any
    site still needs its first, exact-amax quantisation (the per-weight path does that)."""
    for w in ws:
        sites = getattr(w, "_ringdp_fp8", None)
        hist = sites[2] if sites is not None else None
        if hist is None or hist.numel() != 1 + C.fp8_delayed_slots(w.shape[0], w.shape[1]):
            return False
    hists = []
    for w in ws:
        hist, init, roll = _site(w, 2, 1 + C.fp8_delayed_slots(w.shape[0], w.shape[1]), w.device)
        if roll:
            C.fp8_roll(hist)
        hists.append(hist)
    flat = C.fp8_quantize_weights([w.detach().contiguous() for w in ws], hists)
    for i, w in enumerate(ws):
        _FP8_WEIGHTS[id(w)] = (w, tuple(flat[3 * i:3 * i + 3]))
    return True


def _quant_weight(w: torch.Tensor):
    """(q, q^T, scale) of a linear weight: from the forward's batched launch, or quantised here."""
    e = _FP8_WEIGHTS.get(id(w))
    if e is not None and e[0] is w:
        return e[1]
    return _quant_act(_bf16(w), w, 2)


def _bf16_t(wb: torch.Tensor) -> torch.Tensor:
    """W^T of a bf16 weight copy: from the forward's cast launch when it made one, else a transpose."""
    e = _BF16_WEIGHTS_T.pop(id(wb), None)
    return e[1] if e is not None and e[0] is wb else C.transpose_bf16(wb)


def _bf16(w: torch.Tensor) -> torch.Tensor:
    cached = _BF16_WEIGHTS.get(id(w))
    if cached is not None:
        return cached
    out = torch.empty(w.shape, device=w.device, dtype=torch.bfloat16)
    C.cast_copy(out, w.detach().contiguous())
    return out


def _splits(k: int, m: int = 128, n: int = 128, cus: int = 256) -> int:
    """Split-K count for an (m x n) weight-gradient GEMM reducing over k rows: enough workgroups to
    cover the chip twice, but few fp32 partial planes (each is m*n*4 bytes of traffic)."""
    tiles = ((m + 127) // 128) * ((n + 127) // 128)
    want = max(1, (2 * cus + tiles - 1) // tiles)
    return max(1, min(want, k // 256, 32))


class LinearF(torch.autograd.Function):
    """y = act(x W^T + b) [+ residual]; act 0 = identity, 2 = GELU (erf)."""

    @staticmethod
    def forward(ctx, x, w, b, residual, act: int, out_f32: bool):
        M, K = x.shape
        N = w.shape[0]
        if _FP8["on"] and M % 16 == 0 and N % 16 == 0 and K % 16 == 0:
            return _linear_fp8_fwd(ctx, x, w, b, residual, act, out_f32)
        ctx.fp8 = False
        if getattr(x, "_ringdp_q8", None) is not None:
            raise RuntimeError("LinearF: x is an e4m3-only LayerNorm output (LayerNormFork8) but this linear "
                               "is not on the fp8 path")
        Np = (N + 7) // 8 * 8  # the weight-gradient GEMM walks rows of W in 16-B vectors
        wb = _bf16(w)
        bb = b
        if Np != N:
            if residual is not None or act:
                raise ValueError("LinearF: output features must be a multiple of 8 with residual/activation")
            wb = torch.cat([wb, wb.new_zeros(Np - N, K)])
            bb = None if b is None else torch.cat([b.detach(), b.new_zeros(Np - N)])
        pre = torch.empty(M, Np, device=x.device, dtype=torch.bfloat16) if act == 2 else None
        y = C.gemm(x, wb, M, Np, K, K, K, False, False, 1, 0, 0, not out_f32, bb, act, residual, pre).view(M, Np)
        if Np != N:
            y = y[:, :N].contiguous()
        ctx.save_for_backward(x, wb, pre)
        ctx.params = (w, b)
        ctx.cfg = (act, residual is not None, N)
        return y

    @staticmethod
    def backward(ctx, dy):
        if ctx.fp8:
            return _linear_fp8_bwd(ctx, dy)
        x, wb, pre = ctx.saved_tensors
        w, b = ctx.params
        act, has_res, n_out = ctx.cfg
        M, K = x.shape
        N = wb.shape[0]
        if N != n_out:
            dyp = torch.zeros(M, N, device=dy.device, dtype=torch.bfloat16)
            dyp[:, :n_out] = dy
            dy = dyp
        dyb = dy.contiguous() if dy.dtype == torch.bfloat16 else _bf16(dy)
        dz = C.gelu_bwd(dyb, pre) if act == 2 else dyb
        dx = None
        if ctx.needs_input_grad[0]:
            # dX[m][k] = sum_n dz[m][n] W[n][k]: W^T K-contiguous (from the forward's cast launch) for the
            # phased 256x256 kernel, or W read row-contiguously (RINGDP_DGRAD_WT=0)
            if _DGRAD_WT:
                dx = C.gemm(dz, _bf16_t(wb), M, K, N, N, N, False, False).view(M, K)
            else:
                dx = C.gemm(dz, wb, M, K, N, N, K, False, True).view(M, K)
        dw = db = None
        if ctx.needs_input_grad[1]:
            # dW[n][k] = sum_m dz[m][n] x[m][k]:  A = dz^T, B = x^T (both row-contiguous), split over m
            dw = grad_buffer(w)
            if N == n_out:
                C.gemm_splitk_f32(dz, x, N, K, M, N, K, True, True, _splits(M, N, K), dw)
            else:
                full_w = torch.empty(N, K, device=dy.device, dtype=torch.float32)
                C.gemm_splitk_f32(dz, x, N, K, M, N, K, True, True, _splits(M, N, K), full_w)
                dw.copy_(full_w[:n_out])
        if b is not None and ctx.needs_input_grad[2]:
            db = grad_buffer(b)
            part = getattr(dy, "_ringdp_colsum_part", None)  # per-batch column sums from the attention backward
            if part is not None and act != 2 and N == n_out and part.shape[1] == N:
                C.rowsum_f32(part, db)
            elif N == n_out:
                C.colsum_f32(dz, db)  # bias gradient = column sums of dz (one read of dz)
            else:
                full = torch.empty(N, device=dy.device, dtype=torch.float32)
                C.colsum_f32(dz, full)
                db.copy_(full[:n_out])
        dres = dyb if has_res and ctx.needs_input_grad[3] else None
        return dx, dw, db, dres, None, None


_FP8_DELAYED = os.environ.get("RINGDP_FP8_DELAYED", "1") == "1"
_FP8_BATCH_ROLL = os.environ.get("RINGDP_FP8_BATCH_ROLL", "1") == "1"


class _RollSet:
    """The delayed-scaling sites of one device, rolled together: the first quantisation of a step that
    finds its site already used since the last roll rolls EVERY site in one launch
    (``fp8_roll_many``, one workgroup per site) instead of one ``amax_roll`` launch per quantisation
    (ViT-B/16: 144 launches of ~5 us per step).  Each site's scale still comes from its own previous
    call's tile maxima; a roll of a site not called since is a no-op (same maxima, same result)."""

    def __init__(self):
        self.sites = []          # (weakref to the weight, slot): the history lives on the weight
        self.table = None        # (int64 pointers, int32 tile counts) of the current history tensors
        self.dirty = True

    def register(self, w, slot):
        self._prune()
        if not any(r() is w and k == slot for r, k in self.sites):
            self.sites.append((weakref.ref(w), slot))
        self.dirty = True

    def _prune(self):
        """Forget the sites of weights that no longer exist (models torn down between evals / sweeps)."""
        alive = [(r, k) for r, k in self.sites if r() is not None]
        if len(alive) != len(self.sites):
            self.sites = alive
            self.dirty = True

    def roll(self, device):
        self._prune()
        if self.dirty:
            live = [h for h in (r()._ringdp_fp8[k] for r, k in self.sites) if h is not None]
            ptrs = torch.tensor([h.data_ptr() for h in live], dtype=torch.int64)
            ns = torch.tensor([h.numel() - 1 for h in live], dtype=torch.int32)
            self.table = (ptrs.to(device), ns.to(device), live)
            self.dirty = False
        C.fp8_roll_many(self.table[0], self.table[1])
        for r, k in self.sites:
            w = r()
            if w is not None:
                w._ringdp_fp8_used[k] = False


_ROLLS = {}


def _site(w: torch.Tensor, slot: int, n: int, device) -> Tuple[torch.Tensor, bool, bool]:
    """The delayed-scaling history of site ``slot`` on weight ``w`` ([amax to scale by, n - 1 tile maxima of
    the last call]): returns (hist, init, roll_here).  Slots: 0 the linear's input, 1 its output gradient,
    2 its weight, 3 (on fc2) the input fc1's epilogue quantises, 4 (on fc1) the output gradient fc2's
    data-gradient epilogue quantises, 5 the input a LayerNorm forward quantises (LayerNormFork8).  ``init``: first use (or a new shape) - the caller measures an exact
    amax.  ``roll_here``: the caller rolls this site itself (per-site mode, or a capture that cannot
    upload the batched roll's table); otherwise the batched roll already ran when needed."""
    sites = getattr(w, "_ringdp_fp8", None)
    if sites is None:
        sites = w._ringdp_fp8 = [None] * 6
        w._ringdp_fp8_used = [False] * 6
    used = w._ringdp_fp8_used
    hist = sites[slot]
    init = hist is None or hist.numel() != n
    if init:
        hist = sites[slot] = torch.zeros(n, device=device, dtype=torch.float32)
    if not _FP8_BATCH_ROLL:
        return hist, init, not init
    rs = _ROLLS.setdefault(device, _RollSet())
    if init:
        rs.register(w, slot)
    elif used[slot]:
        if rs.dirty and torch.cuda.is_current_stream_capturing():  # no table upload inside a capture
            return hist, init, True
        rs.roll(device)
    used[slot] = True
    return hist, init, False


def _quant_act(t: torch.Tensor, w: torch.Tensor, slot: int, colsum: Optional[torch.Tensor] = None,
               gelu_pre: Optional[torch.Tensor] = None):
    """fp8 quantisation of an activation (slot 0: the linear's input x), output gradient (slot 1: dz) or
    the bf16 copy of the weight (slot 2) with per-site delayed scaling (TransformerEngine-style, history length 1), state kept on the weight:
    the first quantisation of a site measures its exact amax; later ones scale by the amax the previous
    step measured (values clamped to the e4m3 range) and record the current one inside the same pass,
    which removes the separate amax pass over the tensor.  ``gelu_pre``: quantise ``t * GELU'(gelu_pre)``
    instead (the GELU backward done inside the quantisation pass).  The rolls of all sites run as one
    launch per step (``_RollSet``)."""
    if not _FP8_DELAYED:
        return C.fp8_quantize_both(t if gelu_pre is None else C.gelu_bwd(t, gelu_pre))
    hist, init, roll = _site(w, slot, 1 + C.fp8_delayed_slots(t.shape[0], t.shape[1]), t.device)
    return C.fp8_quantize_both_delayed(t, hist, init, colsum, gelu_pre, roll=roll)


_FP8_MLP_FUSED = os.environ.get("RINGDP_FP8_MLP_FUSED", "1") == "1"


def fp8_mlp_fusable(M: int, D: int, Hd: int) -> bool:
    """MLPF8 needs whole 16-row / 16-column e4m3 pieces and whole 128-byte k-steps (K = D)."""
    return _FP8_MLP_FUSED and _FP8_DELAYED and M % 16 == 0 and Hd % 16 == 0 and D % 128 == 0


def _epilogue_site(w, slot, M, N, device, exact_from: int):
    """History of an epilogue-quantised site; on its first use the caller takes the unfused path, whose
    quant_t site ``exact_from`` on the same weight measures the exact amax this one then starts from."""
    hist, init, roll = _site(w, slot, 1 + C.gemm_fp8_q8_slots(M, N), device)
    if roll:
        C.fp8_roll(hist)
    return hist, init


class MLPF8(torch.autograd.Function):
    """The transformer MLP ``y = fc2(GELU(fc1(h))) + residual`` in e4m3 with the [tokens, 3072] tensors
    quantised by the GEMM epilogues that produce them (ringdp's fp8 256x256 kernel, ``ep.q8``):
      forward   fc1's epilogue applies bias + GELU, stores the bf16 pre-activation (for the backward) and
                writes GELU(.) as e4m3 row-major (fc2's A) and transposed (fc2's weight gradient) - the bf16
                activation never reaches memory and fc2's input needs no quant_t pass;
      backward  fc2's data-gradient epilogue applies the GELU backward and writes dz1 as e4m3 (both
                orientations) plus its column sums (fc1's bias gradient) - no bf16 dz1, no quant_t pass.
    Scales are delayed (the sites' previous amax, rolled once per step) exactly like the quant_t sites;
    the first call of each epilogue site runs the unfused path to measure an exact amax."""

    @staticmethod
    def forward(ctx, h, w1, b1, w2, b2, residual):
        M, D = h.shape
        Hd = w1.shape[0]
        hq, hqt, sh = _q8_of(h, w1)
        w1q, w1qt, sw1 = _quant_weight(w1)
        pre = torch.empty(M, Hd, device=h.device, dtype=torch.bfloat16)
        hist3, init3 = _epilogue_site(w2, 3, M, Hd, h.device, 0)
        if init3:
            a = C.gemm_fp8(hq, w1q, sh, sw1, M, Hd, D, True, b1, 2, None, pre)
            aq, aqt, sa = _quant_act(a, w2, 0)
            hist3[:1].copy_(w2._ringdp_fp8[0][:1])
        else:
            aq, aqt, sa = C.gemm_fp8_quant_out(hq, w1q, sh, sw1, M, Hd, D, b1, 2, pre, hist3)
        w2q, w2qt, sw2 = _quant_weight(w2)
        y = C.gemm_fp8(aq, w2q, sa, sw2, M, D, Hd, True, b2, 0, residual)
        ctx.save_for_backward(hqt, sh, w1qt, sw1, pre, aqt, sa, w2qt, sw2)
        ctx.params = (w1, b1, w2, b2)
        ctx.dims = (M, D, Hd)
        ctx.has_res = residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        hqt, sh, w1qt, sw1, pre, aqt, sa, w2qt, sw2 = ctx.saved_tensors
        w1, b1, w2, b2 = ctx.params
        M, D, Hd = ctx.dims
        n = ctx.needs_input_grad
        dyb = dy.contiguous() if dy.dtype == torch.bfloat16 else _bf16(dy)
        db2 = grad_buffer(b2) if n[4] else None
        dyq, dyqt, sdy = _quant_act(dyb, w2, 1, db2)
        dw2 = None
        if n[3]:
            dw2 = grad_buffer(w2)
            C.gemm_fp8_splitk_f32(dyqt, aqt, sdy, sa, D, Hd, M, _splits(M, D, Hd), dw2)
        db1 = grad_buffer(b1) if n[2] else None
        hist4, init4 = _epilogue_site(w1, 4, M, Hd, dy.device, 1)
        if init4:
            da = C.gemm_fp8(dyq, w2qt, sdy, sw2, M, Hd, D, True)
            dzq, dztq, sdz = _quant_act(da, w1, 1, db1, pre)
            hist4[:1].copy_(w1._ringdp_fp8[1][:1])
        else:
            dzq, dztq, sdz = C.gemm_fp8_quant_out(dyq, w2qt, sdy, sw2, M, Hd, D, None, 3, pre, hist4, db1)
        dw1 = None
        if n[1]:
            dw1 = grad_buffer(w1)
            C.gemm_fp8_splitk_f32(dztq, hqt, sdz, sh, Hd, D, M, _splits(M, Hd, D), dw1)
        dh = C.gemm_fp8(dzq, w1qt, sdz, sw1, M, D, Hd, True) if n[0] else None
        dres = dyb if ctx.has_res and n[5] else None
        return dh, dw1, db1, dw2, db2, dres


def _linear_fp8_fwd(ctx, x, w, b, residual, act, out_f32):
    M, K = x.shape
    N = w.shape[0]
    xq, xtq, sx = _q8_of(x, w)           # row-major for this GEMM, transposed for the weight grad
    wq, wtq, sw = _quant_weight(w)       # ... and for the data grad
    pre = torch.empty(M, N, device=x.device, dtype=torch.bfloat16) if act == 2 else None
    y = C.gemm_fp8(xq, wq, sx, sw, M, N, K, not out_f32, b, act, residual, pre)
    ctx.fp8 = True
    ctx.save_for_backward(xtq, sx, wtq, sw, pre)
    ctx.shape = (M, K)
    ctx.params = (w, b)
    ctx.cfg = (act, residual is not None, N)
    return y


def _linear_fp8_bwd(ctx, dy):
    xtq, sx, wtq, sw, pre = ctx.saved_tensors
    w, b = ctx.params
    act, has_res, N = ctx.cfg
    M, K = ctx.shape
    dyb = dy.contiguous() if dy.dtype == torch.bfloat16 else _bf16(dy)
    dx = dw = None
    want_db = b is not None and ctx.needs_input_grad[2]
    db = grad_buffer(b) if want_db and _FP8_DELAYED else None  # column sums of dz from the quantisation pass
    # dz = dy * GELU'(pre) is formed inside the quantisation pass (delayed scaling) - never stored in bf16
    fuse = act == 2 and _FP8_DELAYED
    dz = dyb if act != 2 or fuse else C.gelu_bwd(dyb, pre)
    dzq, dztq, sdz = _quant_act(dz, w, 1, db, pre if fuse else None)  # [M][N] data grad, [N][M] weight grad
    if ctx.needs_input_grad[0]:
        dx = C.gemm_fp8(dzq, wtq, sdz, sw, M, K, N, True)
    if ctx.needs_input_grad[1]:
        dw = grad_buffer(w)
        C.gemm_fp8_splitk_f32(dztq, xtq, sdz, sx, N, K, M, _splits(M, N, K), dw)
    if want_db and db is None:
        db = grad_buffer(b)
        C.colsum_f32(dz, db)
    dres = dyb if has_res and ctx.needs_input_grad[3] else None
    return dx, dw, db, dres, None, None


class MLPF(torch.autograd.Function):
    """The transformer MLP ``y = fc2(GELU(fc1(h))) + residual`` as one Function (bf16 path), so that
    the backward runs the GELU derivative inside fc2's data-gradient GEMM epilogue (ringdp's act-3
    epilogue) instead of a separate pass over the [tokens, 3072] gradient
    (gelu_bwd: 79 us per ViT-B/16 block)."""

    @staticmethod
    def forward(ctx, h, w1, b1, w2, b2, residual):
        M, D = h.shape
        Hd = w1.shape[0]
        w1b, w2b = _bf16(w1), _bf16(w2)
        pre = torch.empty(M, Hd, device=h.device, dtype=torch.bfloat16)
        a = C.gemm(h, w1b, M, Hd, D, D, D, False, False, 1, 0, 0, True, b1, 2, None, pre).view(M, Hd)
        y = C.gemm(a, w2b, M, D, Hd, Hd, Hd, False, False, 1, 0, 0, True, b2, 0, residual).view(M, D)
        ctx.save_for_backward(h, w1b, w2b, pre, a)
        ctx.params = (w1, b1, w2, b2)
        ctx.has_res = residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        h, w1b, w2b, pre, a = ctx.saved_tensors
        w1, b1, w2, b2 = ctx.params
        M, D = h.shape
        Hd = w1b.shape[0]
        dy_in = dy
        dy = dy.contiguous() if dy.dtype == torch.bfloat16 else _bf16(dy)
        db1 = grad_buffer(b1)
        # d(fc1 output) = (dy W2) * GELU'(pre): the GELU backward rides in the GEMM epilogue (act 3), and so do
        # the column sums of the stored dz1 (fc1's bias gradient: no separate pass over [tokens, 3072])
        if _DGRAD_WT:
            dz1 = C.gemm(dy, _bf16_t(w2b), M, Hd, D, D, D, False, False, 1, 0, 0, True, None, 3, None,
                         pre, colsum=db1).view(M, Hd)
        else:
            dz1 = C.gemm(dy, w2b, M, Hd, D, D, Hd, False, True, 1, 0, 0, True, None, 3, None, pre,
                         colsum=db1).view(M, Hd)
        dw2, db2 = grad_buffer(w2), grad_buffer(b2)
        C.gemm_splitk_f32(dy, a, D, Hd, M, D, Hd, True, True, _splits(M, D, Hd), dw2)
        part = getattr(dy_in, "_ringdp_colsum_part", None)  # from the LayerNorm backward that produced dy
        if part is not None and part.shape[1] == D:
            C.rowsum_f32(part, db2)
        else:
            C.colsum_f32(dy, db2)
        dw1 = grad_buffer(w1)
        C.gemm_splitk_f32(dz1, h, Hd, D, M, Hd, D, True, True, _splits(M, Hd, D), dw1)
        dh = None
        if ctx.needs_input_grad[0]:
            if _DGRAD_WT:
                dh = C.gemm(dz1, _bf16_t(w1b), M, D, Hd, Hd, Hd, False, False).view(M, D)
            else:
                dh = C.gemm(dz1, w1b, M, D, Hd, Hd, D, False, True).view(M, D)
        dres = dy if ctx.has_res else None
        return dh, dw1, db1, dw2, db2, dres


class LayerNormFork(torch.autograd.Function):
    """LayerNorm that also hands its input on as the residual stream: ``y, x_id = LayerNormFork(x)``.
    The residual's gradient then arrives here and the LayerNorm backward kernel adds it to dx (its
    ``dres`` input) instead of autograd summing the two gradients of ``x`` in a separate pass."""

    @staticmethod
    def forward(ctx, x, w, b, eps: float):
        y, stats = C.layernorm_fwd(x, w, b, eps)
        ctx.save_for_backward(x, stats)
        ctx.params = (w, b)
        return y, x

    @staticmethod
    def backward(ctx, dy, dres):
        x, stats = ctx.saved_tensors
        w, b = ctx.params
        if dy is None:
            return dres, None, None, None
        dw, db = grad_buffer(w), grad_buffer(b)
        res = dres.contiguous() if dres is not None else None
        if _FP8["on"] or not _LN_COLSUM:  # (fp8 linears take their bias gradients from the quantisation pass)
            dx = C.layernorm_bwd(dy.contiguous(), x, stats, w, res, dw, db)
        else:
            # dx is the output gradient of the linear that produced x (attention proj / fc2, residual fused):
            # its bias gradient's column sums come from this kernel instead of a pass over dx
            dx, part = C.layernorm_bwd_colsum(dy.contiguous(), x, stats, w, res, dw, db)
            dx._ringdp_colsum_part = part
        return dx, dw, db, None


_FP8_LN_Q8 = os.environ.get("RINGDP_FP8_LN_Q8", "1") == "1"


class LayerNormFork8(torch.autograd.Function):
    """LayerNormFork for an fp8 consumer: the forward writes the normalised rows as e4m3 (row-major and
    transposed, delayed scale of the consumer weight's site 5) instead of bf16, so the consumer linear needs
    no quantisation pass.  The returned ``y`` is an unwritten placeholder carrying the e4m3 triple
    (``_ringdp_q8``), read only by LinearF / MLPF8; the backward is LayerNormFork's.  The first call of a site
    runs the bf16 LayerNorm and measures the exact amax."""

    @staticmethod
    def forward(ctx, x, w, b, eps: float, consumer_w):
        rows = x.shape[0]
        hist, init, roll = _site(consumer_w, 5, 1 + C.layernorm_q8_slots(rows), x.device)
        ctx.params = (w, b)
        if init:
            y, stats = C.layernorm_fwd(x, w, b, eps)
            hist[:1].copy_(y.float().abs().amax().reshape(1))
            ctx.save_for_backward(x, stats)
            return y, x
        if roll:
            C.fp8_roll(hist)
        stats, q, qt, scale = C.layernorm_fwd_q8(x, w, b, eps, hist)
        ctx.save_for_backward(x, stats)
        y = torch.empty_like(x)
        y._ringdp_q8 = (q, qt, scale)
        return y, x

    @staticmethod
    def backward(ctx, dy, dres):
        dx, dw, db, _ = LayerNormFork.backward(ctx, dy, dres)
        return dx, dw, db, None, None


def _fork8_ok(x, consumer_w) -> bool:
    """LayerNormFork8's placeholder ``y`` is only valid if the consumer takes the fp8 path: LinearF's
    condition (rows, D and the consumer's out_features multiples of 16) and the e4m3 LayerNorm kernel's
    D <= 2048."""
    rows, d = x.shape[0], x.shape[-1]
    return x.dim() == 2 and rows % 16 == 0 and d % 16 == 0 and d <= 2048 and consumer_w.shape[0] % 16 == 0 \
        and consumer_w.shape[-1] == d


def layernorm_fork(x, ln, consumer_w):
    """``y, x_id`` of LayerNormFork, or of LayerNormFork8 when the consumer is an fp8 linear."""
    if _FP8["on"] and _FP8_LN_Q8 and _FP8_DELAYED and _fork8_ok(x, consumer_w):
        return LayerNormFork8.apply(x, ln.weight, ln.bias, ln.eps, consumer_w)
    return LayerNormFork.apply(x, ln.weight, ln.bias, ln.eps)


def _q8_of(x, w, slot=0):
    """(q, q^T, scale) of an fp8 GEMM input: from the producing LayerNorm (LayerNormFork8) or quantised here."""
    e = getattr(x, "_ringdp_q8", None)
    if e is not None:
        return e
    return _quant_act(x, w, slot)


class LayerNormF(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps: float):
        y, stats = C.layernorm_fwd(x, w, b, eps)
        ctx.save_for_backward(x, stats)
        ctx.params = (w, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, stats = ctx.saved_tensors
        w, b = ctx.params
        dw, db = grad_buffer(w), grad_buffer(b)
        dx = C.layernorm_bwd(dy.contiguous(), x, stats, w, None, dw, db)
        return dx, dw, db, None


def _tp(t: int) -> int:
    return (t + 15) // 16 * 16


class AttentionF(torch.autograd.Function):
    """Multi-head self-attention core on the packed qkv rows [B*T, 3*D] -> [B*T, D]."""

    @staticmethod
    def forward(ctx, qkv, B: int, T: int, H: int):
        Tp = _tp(T)
        Dh = qkv.shape[1] // (3 * H)
        if Dh == 64 and Tp <= 256 and not _ATTN_UNFUSED and not _ATTN_BWD_GEMMS:
            # fused kernels straight on the projection rows: no head-major split / merge passes
            scale = 1.0 / math.sqrt(Dh)
            p, out = C.attn_fwd_rows(qkv, B, T, H, scale, _ATTN_RECOMPUTE)  # p: P, or the log-sum-exp
            ctx.save_for_backward(qkv, p)
            ctx.cfg = (B, T, H, Tp, scale)
            ctx.rows = True
            return out
        ctx.rows = False
        q, k, v = C.qkv_split(qkv, B, T, H, Tp)
        BH, _, Dh = q.shape
        scale = 1.0 / math.sqrt(Dh)
        if Dh == 64 and Tp <= 256 and not _ATTN_UNFUSED:
            # one kernel: S stays in registers, P (for the backward) and O are written
            p, o = C.attn_fwd(q, k, v, T, scale)
        else:
            # S = Q K^T (fp32), P = softmax(scale * S) over the T real keys
            s = C.gemm(q, k, Tp, Tp, Dh, Dh, Dh, False, False, BH, Tp * Dh, Tp * Dh, False)
            p = C.softmax_fwd(s, T, scale)
            # O = P V:  A = P (K-contiguous over keys), B = V^T (row-contiguous: element (d, t) = V[t][d])
            o = C.gemm(p, v, Tp, Dh, Tp, Tp, Dh, False, True, BH, Tp * Tp, Tp * Dh, True)
        ctx.save_for_backward(q, k, v, p)
        ctx.cfg = (B, T, H, Tp, scale)
        return C.heads_to_rows(o.view(BH, Tp, Dh), B, T)

    @staticmethod
    def backward(ctx, dout):
        if ctx.rows:
            qkv, p = ctx.saved_tensors
            B, T, H, Tp, scale = ctx.cfg
            if p.dtype == torch.float32 and not _FP8["on"]:
                # the kernels also sum their dq / dk / dv rows per batch: the qkv projection's bias gradient is
                # then one [B, 3D] -> [3D] reduction in LinearF's backward instead of a pass over dqkv
                part = torch.empty(B, qkv.shape[1], device=qkv.device, dtype=torch.float32)
                dqkv = C.attn_bwd_rows(dout.contiguous(), qkv, p, B, T, H, scale, part)
                dqkv._ringdp_colsum_part = part
                return dqkv, None, None, None
            return C.attn_bwd_rows(dout.contiguous(), qkv, p, B, T, H, scale), None, None, None
        q, k, v, p = ctx.saved_tensors
        B, T, H, Tp, scale = ctx.cfg
        BH, _, Dh = q.shape
        do = C.rows_to_heads(dout.contiguous(), B, T, H, Tp)
        if Dh == 64 and Tp <= 256 and not _ATTN_UNFUSED and not _ATTN_BWD_GEMMS:
            # two fused kernels: query side (dS in registers, dQ) and key side (dK, dV), written
            # straight into the qkv gradient rows
            return C.attn_bwd(do, q, k, v, p, B, T, H, scale), None, None, None
        # dP = dO V^T (fp32) -> dS = scale * P * (dP - rowsum(dP * P))
        if Dh == 64 and Tp <= 256 and not _ATTN_UNFUSED:
            ds = C.attn_bwd_ds(do, v, p, scale)  # dP stays in registers
        else:
            dp = C.gemm(do, v, Tp, Tp, Dh, Dh, Dh, False, False, BH, Tp * Dh, Tp * Dh, False)
            ds = C.softmax_bwd(p, dp, T, scale)
        # dQ = dS K ; dK = dS^T Q ; dV = P^T dO
        dq = C.gemm(ds, k, Tp, Dh, Tp, Tp, Dh, False, True, BH, Tp * Tp, Tp * Dh, True)
        dk = C.gemm(ds, q, Tp, Dh, Tp, Tp, Dh, True, True, BH, Tp * Tp, Tp * Dh, True)
        dv = C.gemm(p, do, Tp, Dh, Tp, Tp, Dh, True, True, BH, Tp * Tp, Tp * Dh, True)
        dqkv = C.qkv_merge(dq.view(BH, Tp, Dh), dk.view(BH, Tp, Dh), dv.view(BH, Tp, Dh), B, T)
        return dqkv, None, None, None


class PatchTokensF(torch.autograd.Function):
    """Patch embedding (stride = kernel conv as one GEMM over the patch rows) + class token +
    position embedding -> token rows [B*T, D]."""

    @staticmethod
    def forward(ctx, x, w, b, cls, pos, patch: int):
        Bn = x.shape[0]
        D = w.shape[0]
        rows = C.patchify(x.contiguous(), patch)  # [B*NP, C*P*P]
        wb = _bf16(w.reshape(D, -1))
        emb = C.gemm(rows, wb, rows.shape[0], D, rows.shape[1], rows.shape[1], rows.shape[1], False, False, 1, 0, 0,
                     True, b)
        NP = rows.shape[0] // Bn
        tokens = C.assemble_tokens(emb.view(Bn, NP, D), cls.reshape(-1), pos.reshape(-1))
        ctx.save_for_backward(rows)
        ctx.params = (w, b, cls, pos)
        ctx.cfg = (Bn, NP, D)
        return tokens.view(Bn * (NP + 1), D)

    @staticmethod
    def backward(ctx, dtok):
        (rows,) = ctx.saved_tensors
        w, b, cls, pos = ctx.params
        Bn, NP, D = ctx.cfg
        dpos, dcls = grad_buffer(pos), grad_buffer(cls)
        demb = C.assemble_tokens_bwd(dtok.contiguous().view(Bn, NP + 1, D), dpos, dcls).view(Bn * NP, D)
        M, K = rows.shape
        dw = grad_buffer(w)
        C.gemm_splitk_f32(demb, rows, D, K, M, D, K, True, True, _splits(M, D, K), dw)
        db = grad_buffer(b)
        C.colsum_f32(demb.contiguous(), db)
        return None, dw, db, dcls, dpos, None


class ClassRowsF(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, B: int, T: int):
        ctx.cfg = (B, T)
        return C.cls_rows(x, B, T, False)

    @staticmethod
    def backward(ctx, dy):
        B, T = ctx.cfg
        return C.cls_rows(dy.contiguous().to(torch.bfloat16), B, T, True).view(B * T, -1), None, None


def linear(x, lin, act: int = 0, residual: Optional[torch.Tensor] = None, out_f32: bool = False):
    return LinearF.apply(x, lin.weight, lin.bias, residual, act, out_f32)
