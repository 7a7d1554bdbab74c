"""SGD with momentum / dampening / nesterov / weight decay / maximize.

Math parity: ``torch/optim/sgd.py:343-380``, the optimizer of both
reference workloads (``ref/launch_dist.py:59``: plain SGD lr 1e-4; ``ref/example_mp.py:84-90``:
lr 0.02, momentum 0.9, wd 1e-4, nesterov).

GPU paths (one launch per step, no per-tensor foreach chains):
* flat  - when the parameters were flattened by ringdp's DDP into one buffer whose layout matches
          the gradient bucket buffer, a single float4 kernel updates the entire range (for the
          ConvNet it also writes next step's bf16 MFMA weight fragments: no pack launch per forward);
* multi - otherwise one multi-tensor kernel over a pointer table.
CPU: the same math with ATen foreach ops.

``lr`` may be a 0-dim float32 CUDA tensor: the kernel then reads it from device memory, so a
captured hipGraph step picks up learning-rate schedule changes without re-capture.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
from torch.optim.optimizer import Optimizer

from .._native import C
from ..utils import tracing as _tracing


# RINGDP_CN_PACK_IN_SGD=0: the ConvNet forward packs its weights itself every step (A/B measurements)
_PACK_IN_SGD = os.environ.get("RINGDP_CN_PACK_IN_SGD", "1") != "0"


def _pack_target(params):
    """(state, flat offsets, weights) when the flat step can keep one model's packed weight fragments current
    (ringdp.ops.convnet.PackState: all 4 ConvNet weights in this group, their fragments built once)."""
    if not _PACK_IN_SGD:
        return None
    st, offs, ws = None, {}, {}
    for p in params:
        t = getattr(p, "_ringdp_pack", None)
        if t is None:
            continue
        if st is not None and t[0] is not st:
            return None
        st = t[0]
        offs[t[1]] = p._ringdp_flat[2]
        ws[t[1]] = p
    if st is None or st.buf is None or sorted(offs) != [0, 1, 2, 3]:
        return None
    return st, [offs[i] for i in range(4)], tuple(ws[i] for i in range(4))


def _invalidate_packs(params):
    """The step's kernels changed weights without bumping their versions: their fragments are stale."""
    for p in params:
        t = getattr(p, "_ringdp_pack", None)
        if t is not None:
            t[0].invalidate()


class SGD(Optimizer):
    def __init__(self, params, lr=1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, *, maximize: bool = False,
                 foreach: Optional[bool] = None, differentiable: bool = False, fused: Optional[bool] = None):
        if isinstance(lr, float) and lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if momentum < 0.0:
            raise ValueError(f"Invalid momentum value: {momentum}")
        if weight_decay < 0.0:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        if differentiable:
            raise NotImplementedError("ringdp.optim.SGD: differentiable=True is not supported")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, maximize=maximize)
        super().__init__(params, defaults)
        self._flat_cache = {}
        self._multi_cache = {}

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        # drop the fused-kernel layouts: the next step re-adopts the loaded momentum buffers
        self._flat_cache = {}
        self._multi_cache = {}

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _hyper(group) -> "C.SgdHyper":
        h = C.SgdHyper()
        lr = group["lr"]
        h.lr = float(lr) if not torch.is_tensor(lr) else 0.0
        h.momentum = float(group["momentum"])
        h.dampening = float(group["dampening"])
        h.weight_decay = float(group["weight_decay"])
        h.nesterov = bool(group["nesterov"])
        h.maximize = bool(group["maximize"])
        return h

    def _flat_layout(self, group, params):
        """If every param of the group is a view into one DDP-flattened buffer whose grads are
        the matching bucket views, return (flat_param, flat_grad, flat_momentum or None)."""
        metas = [getattr(p, "_ringdp_flat", None) for p in params]
        if not params or any(m is None for m in metas):
            return None
        fp, fg = metas[0][0], metas[0][1]
        if any(m[0] is not fp or m[1] is not fg for m in metas):
            return None
        if len(params) != metas[0][3]:  # must cover every parameter of the buffer
            return None
        for p, m in zip(params, metas):
            off = m[2]
            if p.grad is None or p.grad.data_ptr() != fg.data_ptr() + off * fg.element_size():
                return None
            if p.data_ptr() != fp.data_ptr() + off * fp.element_size():
                return None
        key = (fp.data_ptr(), id(group))
        mom = None
        first = False
        if group["momentum"] != 0:
            mom = self._flat_cache.get(key)
            if mom is None or mom.numel() != fp.numel():
                mom = torch.zeros_like(fp)
                # Adopt any existing per-parameter momentum (e.g. after load_state_dict).
                have = [self.state[p].get("momentum_buffer") for p in params]
                for p, m, buf in zip(params, metas, have):
                    if buf is not None:
                        mom[m[2]:m[2] + p.numel()].copy_(buf.reshape(-1))
                first = any(b is None for b in have)
                self._flat_cache[key] = mom
            for p, m in zip(params, metas):
                st = self.state[p]
                view = mom[m[2]:m[2] + p.numel()].view_as(p)
                if st.get("momentum_buffer") is None or st["momentum_buffer"].data_ptr() != view.data_ptr():
                    st["momentum_buffer"] = view
        return fp, fg, mom, first

    # ------------------------------------------------------------------ step
    @torch.no_grad()
    @_tracing.annotate("ringdp.SGD.step")
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            if params[0].is_cuda:
                self._step_gpu(group, params)
            else:
                self._step_cpu(group, params)
        return loss

    def _step_gpu(self, group, params):
        h = self._hyper(group)
        lr_t = group["lr"] if torch.is_tensor(group["lr"]) else None
        mom_on = group["momentum"] != 0
        first = mom_on and any(self.state[p].get("momentum_buffer") is None for p in params)
        flat = self._flat_layout(group, params)
        if flat is not None:
            fp, fg, mom, first = flat
            tgt = _pack_target(params)
            if tgt is not None:  # also write the ConvNet's bf16 fragments of the updated weights
                st, offs, ws = tgt
                C.sgd_flat(fp, fg, mom if mom_on else None, h, first, lr_t, None, st.buf, offs)
                st.mark_written(ws)
                return
            C.sgd_flat(fp, fg, mom if mom_on else None, h, first, lr_t, None)
            _invalidate_packs(params)
            return
        _invalidate_packs(params)
        bufs = []
        if mom_on:
            for p in params:
                st = self.state[p]
                if st.get("momentum_buffer") is None:
                    st["momentum_buffer"] = torch.empty_like(p, memory_format=torch.contiguous_format)
                bufs.append(st["momentum_buffer"])
        if not all(p.grad.is_contiguous() and p.is_contiguous() for p in params):
            grads = [p.grad.contiguous() for p in params]
            C.sgd_multi(params, grads, bufs, h, first, lr_t, None)
            return
        # Pointer table cached per (param, grad, buffer) addresses: no host->device copy per step,
        # so the step is hipGraph-capturable once the table exists.
        key = tuple(p.data_ptr() for p in params) + tuple(p.grad.data_ptr() for p in params) + \
            tuple(b.data_ptr() for b in bufs)
        tab = self._multi_cache.get(id(group))
        if tab is None or tab[0] != key:
            dev, nchunks, tbytes = C.sgd_multi_build(params, [p.grad for p in params], bufs, mom_on)
            tab = (key, dev, nchunks, tbytes)
            self._multi_cache[id(group)] = tab
        C.sgd_multi_run(tab[1], tab[2], tab[3], h, first, lr_t, None)

    def _step_cpu(self, group, params):
        lr = float(group["lr"])
        wd, mom, damp = group["weight_decay"], group["momentum"], group["dampening"]
        nesterov, maximize = group["nesterov"], group["maximize"]
        grads = [(-p.grad if maximize else p.grad) for p in params]
        if wd != 0:
            grads = torch._foreach_add(grads, params, alpha=wd)
        if mom != 0:
            bufs = []
            for p, g in zip(params, grads):
                st = self.state[p]
                buf = st.get("momentum_buffer")
                if buf is None:
                    buf = torch.clone(g).detach()
                    st["momentum_buffer"] = buf
                else:
                    buf.mul_(mom).add_(g, alpha=1 - damp)
                bufs.append(buf)
            if nesterov:
                grads = torch._foreach_add(grads, bufs, alpha=mom)
            else:
                grads = bufs
        torch._foreach_add_(params, grads, alpha=-lr)
