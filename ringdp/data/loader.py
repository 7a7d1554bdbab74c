"""Batch loaders.

``DataLoader`` - the host loader the reference scripts use:
``DataLoader(dataset, batch_size=100, shuffle=False, pin_memory=True, sampler=DistributedSampler)``
(ref/mpspawn_dist.py:88, ref/launch_dist.py:73-74) and ``num_workers=4`` for CIFAR
(ref/example_mp.py:74-80).  Batches are produced in sampler order; ``num_workers`` > 0 assembles
batches on a thread pool with a bounded prefetch window (the per-sample transforms are torch ops that
release the GIL), and ``pin_memory`` pins every batch so ``.to(device, non_blocking=True)`` is a
true async H2D copy.

``DeviceLoader`` - the MI355X-first path (§2.4 U15): the whole uint8 dataset lives in HBM (MNIST is
47 MB, CIFAR-10 150 MB against 288 GB), the epoch's sampler indices are one device tensor, and each
batch is ONE HIP launch (``C.gather_augment``: index gather + random crop / flip + ToTensor +
Normalize, writing fp32/bf16 NCHW/NHWC or raw uint8 for the ConvNet, whose first kernel fuses the
normalisation).  No host work per step, so the loop can be captured in a hipGraph.
"""
from __future__ import annotations

import collections
import concurrent.futures as cf
import math
from typing import Callable, Iterator, List, Optional, Sequence

import torch

from .sampler import DistributedSampler
from .transforms import default_collate


class SequentialSampler:
    def __init__(self, data_source):
        self.n = len(data_source)

    def __iter__(self):
        return iter(range(self.n))

    def __len__(self):
        return self.n


class RandomSampler:
    def __init__(self, data_source, generator: Optional[torch.Generator] = None):
        self.n = len(data_source)
        self.generator = generator

    def __iter__(self):
        return iter(torch.randperm(self.n, generator=self.generator).tolist())

    def __len__(self):
        return self.n


class DataLoader:
    def __init__(self, dataset, batch_size: int = 1, shuffle: bool = False, sampler=None,
                 num_workers: int = 0, pin_memory: bool = False, drop_last: bool = False,
                 collate_fn: Optional[Callable] = None, prefetch_factor: int = 2,
                 generator: Optional[torch.Generator] = None):
        if sampler is not None and shuffle:
            # same contract as torch: the sampler owns the order (ref/README.md:170)
            raise ValueError("sampler option is mutually exclusive with shuffle")
        if batch_size < 1:
            raise ValueError("batch_size must be >= 1")
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.sampler = sampler if sampler is not None else (
            RandomSampler(dataset, generator) if shuffle else SequentialSampler(dataset))
        self.num_workers = int(num_workers)
        self.pin_memory = bool(pin_memory) and torch.cuda.is_available()
        self.drop_last = drop_last
        self.collate_fn = collate_fn or default_collate
        self.prefetch = max(1, prefetch_factor) * max(1, self.num_workers)

    def __len__(self) -> int:
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def _batches(self) -> Iterator[List[int]]:
        buf: List[int] = []
        for i in self.sampler:
            buf.append(int(i))
            if len(buf) == self.batch_size:
                yield buf
                buf = []
        if buf and not self.drop_last:
            yield buf

    def _fetch(self, idx: Sequence[int]):
        batch = self.collate_fn([self.dataset[i] for i in idx])
        if self.pin_memory:
            batch = tuple(t.pin_memory() if isinstance(t, torch.Tensor) else t for t in batch)
        return batch

    def __iter__(self):
        if self.num_workers == 0:
            for idx in self._batches():
                yield self._fetch(idx)
            return
        with cf.ThreadPoolExecutor(self.num_workers, thread_name_prefix="ringdp-loader") as ex:
            pending: "collections.deque[cf.Future]" = collections.deque()
            it = self._batches()
            for idx in it:
                pending.append(ex.submit(self._fetch, idx))
                if len(pending) >= self.prefetch:
                    break
            for idx in it:
                yield pending.popleft().result()
                pending.append(ex.submit(self._fetch, idx))
            while pending:
                yield pending.popleft().result()


class DeviceLoader:
    """HBM-resident dataset + one fused gather/augment HIP launch per batch (see module doc)."""

    def __init__(self, dataset, batch_size: int, device, sampler: Optional[DistributedSampler] = None,
                 drop_last: bool = False, crop_padding: int = 0, hflip: bool = False,
                 mean: Optional[Sequence[float]] = None, std: Optional[Sequence[float]] = None,
                 out_dtype: torch.dtype = torch.float32, channels_last: bool = False, seed: int = 0):
        from .._native import C

        self._C = C
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("DeviceLoader needs a GPU device; use DataLoader on CPU")
        self.x = dataset.data.contiguous().to(self.device)
        self.y = dataset.targets.to(torch.int64).contiguous().to(self.device)
        self.batch_size = int(batch_size)
        self.sampler = sampler
        self.drop_last = drop_last
        self.pad = int(crop_padding)
        self.hflip = bool(hflip)
        self.mean = list(mean) if mean is not None else []
        self.std = list(std) if std is not None else []
        if out_dtype == torch.uint8 and (self.mean or self.std):
            raise ValueError("uint8 output carries raw pixels: no mean/std")
        self.out_dtype = out_dtype
        self.nhwc = bool(channels_last)
        self.seed = int(seed)
        self.epoch = 0

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)
        if self.sampler is not None:
            self.sampler.set_epoch(epoch)

    def _epoch_indices(self) -> torch.Tensor:
        if self.sampler is None:
            return torch.arange(self.x.shape[0], device=self.device)
        return torch.tensor(list(iter(self.sampler)), dtype=torch.int64).to(self.device, non_blocking=True)

    def __len__(self) -> int:
        n = len(self.sampler) if self.sampler is not None else int(self.x.shape[0])
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def batch(self, idx: torch.Tensor, step_seed: int):
        """(images, labels) for an explicit device index tensor."""
        return self._C.gather_augment(self.x, self.y, idx, self.pad, self.hflip, self.mean, self.std,
                                      step_seed, self.nhwc, self.out_dtype)

    def __iter__(self):
        idx = self._epoch_indices()
        n = idx.numel()
        stop = n - (n % self.batch_size) if self.drop_last else n
        for k, s in enumerate(range(0, stop, self.batch_size)):
            step_seed = (self.seed * 1000003 + self.epoch) * 1000003 + k
            yield self.batch(idx[s:s + self.batch_size], step_seed)
