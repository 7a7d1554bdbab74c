"""ringdp.nn - loss modules backed by ringdp kernels on GPU (ATen on CPU)."""
from __future__ import annotations

import torch.nn as _nn

from ..ops.loss import cross_entropy


class CrossEntropyLoss(_nn.Module):
    """Drop-in for ``torch.nn.CrossEntropyLoss`` (ref/launch_dist.py:58): fused log-softmax + NLL
    with mean/sum/none reduction, ``ignore_index`` and ``label_smoothing``."""

    def __init__(self, weight=None, size_average=None, ignore_index: int = -100, reduce=None,
                 reduction: str = "mean", label_smoothing: float = 0.0):
        super().__init__()
        if weight is not None:
            raise NotImplementedError("ringdp.nn.CrossEntropyLoss: per-class weights are not supported")
        if size_average is not None or reduce is not None:
            raise NotImplementedError("ringdp.nn.CrossEntropyLoss: legacy size_average/reduce are not supported")
        self.ignore_index = ignore_index
        self.reduction = reduction
        self.label_smoothing = label_smoothing

    def forward(self, input, target):
        return cross_entropy(input, target, self.ignore_index, self.label_smoothing, self.reduction)


__all__ = ["CrossEntropyLoss", "cross_entropy"]
