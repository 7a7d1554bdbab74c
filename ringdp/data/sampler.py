"""DistributedSampler - index-identical to torch.utils.data.DistributedSampler.

Parity: ``torch/utils/data/distributed.py:75-157``, used by the reference at
``ref/mpspawn_dist.py:77-81``, ``ref/launch_dist.py:67-71``, ``ref/example_mp.py:73``.
Semantics kept exactly: ``num_samples = ceil(N / R)`` (or ``ceil((N - R) / R)`` with drop_last
when N % R != 0), ``randperm(N, generator=seed + epoch)`` when shuffling, padding by repeating
the head so every rank gets the same number of samples (DDP needs identical step counts), then
the strided subsample ``indices[rank:total:R]``; ``set_epoch`` reshuffles.

``DeviceDistributedSampler`` yields the same per-rank index stream as an int64 GPU tensor per
batch (for ringdp's on-device loaders: no host round trip per sample).
"""
from __future__ import annotations

import math
from typing import Iterator, Optional, Sized

import torch
from torch.utils.data import Sampler


class DistributedSampler(Sampler):
    def __init__(self, dataset: Sized, num_replicas: Optional[int] = None, rank: Optional[int] = None,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False) -> None:
        if num_replicas is None or rank is None:
            from .. import distributed as dist

            if not dist.is_initialized():
                raise RuntimeError("Requires distributed package to be available")
            if num_replicas is None:
                num_replicas = dist.get_world_size()
            if rank is None:
                rank = dist.get_rank()
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {num_replicas - 1}]")
        self.dataset = dataset
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.drop_last = drop_last
        n = len(self.dataset)
        if self.drop_last and n % self.num_replicas != 0:
            self.num_samples = math.ceil((n - self.num_replicas) / self.num_replicas)
        else:
            self.num_samples = math.ceil(n / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas
        self.shuffle = shuffle
        self.seed = seed

    def _all_indices(self):
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            indices = torch.randperm(n, generator=g).tolist()
        else:
            indices = list(range(n))
        if not self.drop_last:
            padding = self.total_size - len(indices)
            if padding <= len(indices):
                indices += indices[:padding]
            else:
                indices += (indices * math.ceil(padding / len(indices)))[:padding]
        else:
            indices = indices[: self.total_size]
        assert len(indices) == self.total_size
        return indices

    def __iter__(self) -> Iterator[int]:
        indices = self._all_indices()[self.rank : self.total_size : self.num_replicas]
        assert len(indices) == self.num_samples
        return iter(indices)

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch


class DeviceDistributedSampler(DistributedSampler):
    """Same index stream as DistributedSampler, materialised once per epoch on ``device`` and
    sliced into per-batch int64 tensors."""

    def __init__(self, dataset: Sized, batch_size: int, device, **kw):
        super().__init__(dataset, **kw)
        self.batch_size = batch_size
        self.device = torch.device(device)

    def batches(self, drop_last_batch: bool = False):
        idx = torch.tensor(list(super().__iter__()), dtype=torch.long).to(self.device, non_blocking=True)
        n = idx.numel()
        stop = n - (n % self.batch_size) if drop_last_batch else n
        for s in range(0, stop, self.batch_size):
            yield idx[s : s + self.batch_size]

    def num_batches(self, drop_last_batch: bool = False) -> int:
        return self.num_samples // self.batch_size if drop_last_batch else math.ceil(self.num_samples / self.batch_size)
