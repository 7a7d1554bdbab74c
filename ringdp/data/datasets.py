"""Datasets: MNIST / CIFAR-10 readers and deterministic synthetic image sets.

Parity target: the torchvision datasets the reference scripts use:
``MNIST('./data', train=True, download=True, transform=ToTensor+Normalize)``
(ref/launch_dist.py:64-65, ref/mpspawn_dist.py:73-74) and ``CIFAR10(root='./data', train=True)``
(ref/example_mp.py:56-70, ref/example_launch.py:32-46).  torchvision is not part of this stack, so
the on-disk formats are parsed here:

* MNIST: the IDX files (``train-images-idx3-ubyte`` / ``train-labels-idx1-ubyte``, optionally
  ``.gz``) under ``root/MNIST/raw`` or ``root``;
* CIFAR-10: the binary release (``cifar-10-batches-bin/data_batch_{1..5}.bin``), or the python
  release parsed with a restricted unpickler that only admits numpy array reconstruction.

There is no network on MI355X training boxes, so ``download=True`` only checks that the files are
present.  Every dataset keeps its images as one uint8 tensor (N, H, W) or (N, H, W, C) so the
device loader can copy it to HBM once (`ringdp.data.device_loader`).
"""
from __future__ import annotations

import gzip
import io
import os
import pickle
import struct
from typing import Callable, Optional, Sequence, Tuple

import numpy as np
import torch


class ImageDataset:
    """Base: ``data`` uint8 (N, H, W[, C]), ``targets`` int64 (N,)."""

    classes: Sequence[str] = ()

    def __init__(self, data: torch.Tensor, targets: torch.Tensor, transform: Optional[Callable] = None,
                 target_transform: Optional[Callable] = None):
        if data.dtype != torch.uint8:
            raise TypeError(f"image data must be uint8, got {data.dtype}")
        if data.shape[0] != targets.shape[0]:
            raise ValueError("data / targets length mismatch")
        self.data = data
        self.targets = targets.to(torch.int64)
        self.transform = transform
        self.target_transform = target_transform

    def __len__(self) -> int:
        return int(self.data.shape[0])

    def __getitem__(self, i: int) -> Tuple[object, object]:
        img = self.data[i]
        target = int(self.targets[i])
        if self.transform is not None:
            img = self.transform(img)
        if self.target_transform is not None:
            target = self.target_transform(target)
        return img, target


# ------------------------------------------------------------------ MNIST
def _open_maybe_gz(path: str):
    if os.path.exists(path):
        return open(path, "rb")
    if os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rb")
    raise FileNotFoundError(path)


def read_idx(path: str) -> np.ndarray:
    """Parse an IDX file (magic 0x00000803 images / 0x00000801 labels, big-endian dims)."""
    with _open_maybe_gz(path) as f:
        raw = f.read()
    if len(raw) < 4 or raw[0] != 0 or raw[1] != 0:
        raise ValueError(f"{path}: not an IDX file")
    dtype_code, ndim = raw[2], raw[3]
    if dtype_code != 0x08:
        raise ValueError(f"{path}: only unsigned-byte IDX files are supported (code {dtype_code:#x})")
    dims = struct.unpack(">" + "I" * ndim, raw[4:4 + 4 * ndim])
    n = int(np.prod(dims))
    body = raw[4 + 4 * ndim:]
    if len(body) != n:
        raise ValueError(f"{path}: expected {n} bytes of data, found {len(body)}")
    return np.frombuffer(body, dtype=np.uint8).reshape(dims)


def write_idx(path: str, arr: np.ndarray) -> None:
    """Write a uint8 array as IDX (used by tests to build fixture files)."""
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    with open(path, "wb") as f:
        f.write(bytes([0, 0, 0x08, arr.ndim]))
        f.write(struct.pack(">" + "I" * arr.ndim, *arr.shape))
        f.write(arr.tobytes())


class MNIST(ImageDataset):
    classes = tuple(str(i) for i in range(10))
    mean = (0.1307,)
    std = (0.3081,)

    def __init__(self, root: str, train: bool = True, download: bool = False,
                 transform: Optional[Callable] = None, target_transform: Optional[Callable] = None):
        prefix = "train" if train else "t10k"
        cands = [os.path.join(root, "MNIST", "raw"), os.path.join(root, "raw"), root]
        last_err = None
        for d in cands:
            try:
                x = read_idx(os.path.join(d, f"{prefix}-images-idx3-ubyte"))
                y = read_idx(os.path.join(d, f"{prefix}-labels-idx1-ubyte"))
                break
            except FileNotFoundError as e:
                last_err = e
        else:
            hint = " (download=True cannot fetch: no network access)" if download else ""
            raise RuntimeError(f"MNIST {prefix} files not found under {root}{hint}") from last_err
        super().__init__(torch.from_numpy(x.copy()), torch.from_numpy(y.astype(np.int64)), transform,
                         target_transform)


# ------------------------------------------------------------------ CIFAR-10
class _NumpyOnlyUnpickler(pickle.Unpickler):
    """Admits only what the CIFAR python batches contain (dicts of bytes/lists/ndarrays)."""

    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
        ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            mod = __import__(module, fromlist=[name])
            return getattr(mod, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a dataset file")


def _load_cifar_py(path: str):
    with open(path, "rb") as f:
        d = _NumpyOnlyUnpickler(io.BytesIO(f.read()), encoding="bytes").load()
    data = np.asarray(d[b"data"], dtype=np.uint8).reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    labels = np.asarray(d.get(b"labels", d.get(b"fine_labels")), dtype=np.int64)
    return data, labels


def _load_cifar_bin(path: str):
    raw = np.fromfile(path, dtype=np.uint8).reshape(-1, 1 + 3072)
    labels = raw[:, 0].astype(np.int64)
    data = raw[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    return data, labels


class CIFAR10(ImageDataset):
    classes = ("airplane", "automobile", "bird", "cat", "deer", "dog", "frog", "horse", "ship", "truck")
    mean = (0.4914, 0.4822, 0.4465)
    std = (0.2023, 0.1994, 0.2010)

    def __init__(self, root: str, train: bool = True, download: bool = False,
                 transform: Optional[Callable] = None, target_transform: Optional[Callable] = None):
        names = [f"data_batch_{i}" for i in range(1, 6)] if train else ["test_batch"]
        bin_dir = os.path.join(root, "cifar-10-batches-bin")
        py_dir = os.path.join(root, "cifar-10-batches-py")
        parts = []
        if all(os.path.exists(os.path.join(bin_dir, n + ".bin")) for n in names):
            parts = [_load_cifar_bin(os.path.join(bin_dir, n + ".bin")) for n in names]
        elif all(os.path.exists(os.path.join(py_dir, n)) for n in names):
            parts = [_load_cifar_py(os.path.join(py_dir, n)) for n in names]
        else:
            hint = " (download=True cannot fetch: no network access)" if download else ""
            raise RuntimeError(f"CIFAR-10 batches not found under {root}{hint}")
        data = np.concatenate([p[0] for p in parts])
        labels = np.concatenate([p[1] for p in parts])
        super().__init__(torch.from_numpy(np.ascontiguousarray(data)), torch.from_numpy(labels), transform,
                         target_transform)


# ------------------------------------------------------------------ synthetic
class SyntheticImages(ImageDataset):
    """Deterministic uint8 images + labels (same on every rank for the same seed).

    Used by the examples and benchmarks when the real dataset is absent (no network)."""

    def __init__(self, n: int, shape: Tuple[int, ...] = (28, 28), num_classes: int = 10, seed: int = 0,
                 transform: Optional[Callable] = None, target_transform: Optional[Callable] = None):
        g = torch.Generator().manual_seed(seed)
        data = torch.randint(0, 256, (n, *shape), generator=g, dtype=torch.uint8)
        targets = torch.randint(0, num_classes, (n,), generator=g, dtype=torch.int64)
        super().__init__(data, targets, transform, target_transform)


def mnist_or_synthetic(root: str, train: bool = True, transform=None, n_synth: int = 60000, seed: int = 0):
    """Real MNIST when present under ``root``; otherwise a synthetic set of the same shape."""
    try:
        return MNIST(root, train=train, transform=transform), False
    except RuntimeError:
        return SyntheticImages(n_synth if train else 10000, (28, 28), 10, seed, transform), True


def cifar10_or_synthetic(root: str, train: bool = True, transform=None, n_synth: int = 50000, seed: int = 0):
    try:
        return CIFAR10(root, train=train, transform=transform), False
    except RuntimeError:
        return SyntheticImages(n_synth if train else 10000, (32, 32, 3), 10, seed, transform), True
