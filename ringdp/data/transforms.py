"""Host-side image transforms on uint8 tensors (torchvision-compatible semantics).

The reference pipelines:
  W1  ``Compose([ToTensor(), Normalize((0.1307,), (0.3081,))])``       ref/launch_dist.py:64-65
  W2  ``Compose([RandomCrop(32, padding=4), RandomHorizontalFlip(), ToTensor(),
                 Normalize((0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010))])``  ref/example_mp.py:56-70

Images are uint8 tensors, (H, W) for grayscale or (H, W, C) channels-last as stored on disk.
``ToTensor`` produces float32 CHW in [0, 1] exactly like torchvision.  The same transforms run on
the GPU inside the device loader (``ringdp.data.device_loader``: one fused HIP kernel for
gather + crop + flip + normalise); these host versions are the reference semantics and the CPU path.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch


class Compose:
    def __init__(self, transforms: Sequence[Callable]):
        self.transforms = list(transforms)

    def __call__(self, x):
        for t in self.transforms:
            x = t(x)
        return x

    def __repr__(self) -> str:
        return "Compose(" + ", ".join(repr(t) for t in self.transforms) + ")"


def _hwc(img: torch.Tensor) -> torch.Tensor:
    return img.unsqueeze(-1) if img.dim() == 2 else img


class ToTensor:
    """uint8 (H, W[, C]) -> float32 (C, H, W) / 255."""

    def __call__(self, img: torch.Tensor) -> torch.Tensor:
        if img.dtype != torch.uint8:
            raise TypeError("ToTensor expects a uint8 image")
        return _hwc(img).permute(2, 0, 1).contiguous().to(torch.float32).div_(255.0)

    def __repr__(self) -> str:
        return "ToTensor()"


class Normalize:
    def __init__(self, mean: Sequence[float], std: Sequence[float], inplace: bool = False):
        self.mean = tuple(float(m) for m in mean)
        self.std = tuple(float(s) for s in std)
        if any(s == 0 for s in self.std):
            raise ValueError("Normalize: std must be non-zero")
        self.inplace = inplace

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        if not self.inplace:
            t = t.clone()
        m = torch.tensor(self.mean, dtype=t.dtype).view(-1, 1, 1)
        s = torch.tensor(self.std, dtype=t.dtype).view(-1, 1, 1)
        return t.sub_(m).div_(s)

    def __repr__(self) -> str:
        return f"Normalize(mean={self.mean}, std={self.std})"


class RandomCrop:
    """Zero-pad by ``padding`` then crop ``size`` at a uniformly random offset (uint8 HW[C])."""

    def __init__(self, size, padding: int = 0, generator: Optional[torch.Generator] = None):
        self.size = (size, size) if isinstance(size, int) else tuple(size)
        self.padding = int(padding)
        self.generator = generator

    def __call__(self, img: torch.Tensor) -> torch.Tensor:
        x = _hwc(img)
        p = self.padding
        if p:
            x = torch.nn.functional.pad(x.permute(2, 0, 1), (p, p, p, p)).permute(1, 2, 0)
        H, W = x.shape[0], x.shape[1]
        th, tw = self.size
        i = int(torch.randint(0, H - th + 1, (1,), generator=self.generator))
        j = int(torch.randint(0, W - tw + 1, (1,), generator=self.generator))
        out = x[i:i + th, j:j + tw]
        return out.squeeze(-1) if img.dim() == 2 else out.contiguous()

    def __repr__(self) -> str:
        return f"RandomCrop(size={self.size}, padding={self.padding})"


class RandomHorizontalFlip:
    def __init__(self, p: float = 0.5, generator: Optional[torch.Generator] = None):
        self.p = float(p)
        self.generator = generator

    def __call__(self, img: torch.Tensor) -> torch.Tensor:
        if float(torch.rand((), generator=self.generator)) < self.p:
            return img.flip(1).contiguous()
        return img

    def __repr__(self) -> str:
        return f"RandomHorizontalFlip(p={self.p})"


def default_collate(batch: List[Tuple[object, object]]):
    """Stack (image, target) pairs into (images, targets) tensors."""
    xs, ys = zip(*batch)
    x = torch.stack([torch.as_tensor(v) for v in xs])
    y = torch.as_tensor(ys, dtype=torch.int64)
    return x, y
