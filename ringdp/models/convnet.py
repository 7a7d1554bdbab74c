"""MNIST ConvNet (W1) - same parameters / state_dict keys as the reference model.

Reference: ``ref/launch_dist.py:9-41`` (identical copy ``ref/mpspawn_dist.py:11-43``; SURVEY.md
§2.2 R1).  conv1 1->32 k5 p1, MaxPool(2,2); conv2 32->64 k3, MaxPool(2, stride 1); conv3 64->128
k3, MaxPool(2,2); fc1 2048->10.  ``dropout`` is constructed but never called, exactly as in the
reference (quirk §2.8-7), so it is kept for state_dict/API parity only.

GPU: the whole forward/backward runs on ringdp's fused HIP kernels (bf16 activations, fp32
master weights, fp32 accumulation).  CPU: plain ATen ops (BASELINE config #1, gloo/host ring).
Inputs may be float (already normalised, as after ToTensor+Normalize) or raw uint8 pixels, in
which case Normalize((0.1307,), (0.3081,)) is fused into the first kernel.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.convnet import MNIST_MEAN, MNIST_STD, convnet_forward


class ConvNet(nn.Module):
    """``precision``: GPU compute precision - "bf16" (bf16 MFMA, fp32 accumulation and master
    weights; the bench default) or "fp32" (the reference's precision, fp32 MFMA kernels).  The
    CPU path is always fp32 ATen."""

    def __init__(self, precision: str = "bf16"):
        super().__init__()
        if precision not in ("bf16", "fp32"):
            raise ValueError(f"ConvNet: precision must be 'bf16' or 'fp32', got {precision!r}")
        self.precision = precision
        self.relu = nn.ReLU()
        self.conv1 = nn.Conv2d(in_channels=1, out_channels=32, kernel_size=5, stride=1, padding=1)
        self.maxpool1 = nn.MaxPool2d(kernel_size=2, stride=2)
        self.conv2 = nn.Conv2d(in_channels=32, out_channels=64, kernel_size=3, stride=1)
        self.maxpool2 = nn.MaxPool2d(kernel_size=2, stride=1)
        self.conv3 = nn.Conv2d(in_channels=64, out_channels=128, kernel_size=3, stride=1)
        self.maxpool3 = nn.MaxPool2d(kernel_size=2, stride=2)
        self.dropout = nn.Dropout(p=0.5)
        self.fc1 = nn.Linear(in_features=128 * 4 * 4, out_features=10)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            if self.precision == "fp32":
                from ..ops.convnet_fp32 import convnet_forward_fp32

                return convnet_forward_fp32(x, self.conv1, self.conv2, self.conv3, self.fc1)
            return convnet_forward(x, self.conv1, self.conv2, self.conv3, self.fc1)
        return self.reference_forward(x)

    def reference_forward(self, x: torch.Tensor) -> torch.Tensor:
        """ATen math of the reference forward (CPU path and numerics oracle)."""
        if x.dtype == torch.uint8:
            x = (x.float() / 255.0 - MNIST_MEAN) / MNIST_STD
        x = self.maxpool1(self.relu(self.conv1(x)))
        x = self.maxpool2(self.relu(self.conv2(x)))
        x = self.maxpool3(self.relu(self.conv3(x)))
        x = x.reshape(-1, 128 * 4 * 4)
        return self.fc1(x)
