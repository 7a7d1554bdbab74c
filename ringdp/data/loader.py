"""Batch loaders.

``DataLoader`` - the host loader the reference scripts use:
``DataLoader(dataset, batch_size=100, shuffle=False, pin_memory=True, sampler=DistributedSampler)``
(ref/mpspawn_dist.py:88, ref/launch_dist.py:73-74) and ``num_workers=4`` for CIFAR
(ref/example_mp.py:74-80).  Batches are produced in sampler order.  ``num_workers`` > 0 starts that
many worker *processes* (fork context by default, like torch on Linux): batch index lists go out
round-robin on per-worker queues, collated batches come back through shared memory
(torch.multiprocessing), a pin-memory thread in the main process pins them, and the iterator
re-orders them so delivery follows the sampler exactly.  Each worker seeds torch's RNG with
``base_seed + worker_id`` (random transforms differ per worker, reproducibly); a worker exception is
re-raised in the main process with its traceback, a worker that dies is reported by pid.
``worker_mode="thread"`` keeps the lighter thread-pool variant.  ``pin_memory`` pins every batch so
``.to(device, non_blocking=True)`` is a true async H2D copy.

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
import queue
import threading
import traceback
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
                 generator: Optional[torch.Generator] = None, worker_init_fn: Optional[Callable] = None,
                 multiprocessing_context=None, timeout: float = 0, worker_mode: str = "process"):
        if worker_mode not in ("process", "thread"):
            raise ValueError("worker_mode must be 'process' or 'thread'")
        if timeout < 0:
            raise ValueError("timeout option should be non-negative")
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
        self.prefetch_factor = max(1, prefetch_factor)
        self.prefetch = self.prefetch_factor * max(1, self.num_workers)
        self.generator = generator
        self.worker_init_fn = worker_init_fn
        self.multiprocessing_context = multiprocessing_context
        self.timeout = float(timeout)
        self.worker_mode = worker_mode

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

    def _pin(self, batch):
        if not self.pin_memory:
            return batch
        return tuple(t.pin_memory() if isinstance(t, torch.Tensor) else t for t in batch)

    def __iter__(self):
        if self.num_workers == 0:
            for idx in self._batches():
                yield self._fetch(idx)
            return
        if self.worker_mode == "process":
            yield from _MultiProcessIter(self)
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


class _WorkerError:
    def __init__(self, worker_id: int, exc: BaseException):
        self.msg = (f"Caught {type(exc).__name__} in DataLoader worker process {worker_id}.\n"
                    f"Original {traceback.format_exc()}")
        self.exc_type = type(exc)


def _worker_loop(dataset, collate_fn, index_q, result_q, base_seed: int, worker_id: int,
                 num_workers: int, init_fn):
    """Body of one DataLoader worker process (module level: picklable for spawn contexts)."""
    torch.set_num_threads(1)
    torch.manual_seed(base_seed + worker_id)
    import random

    random.seed(base_seed + worker_id)
    try:
        if init_fn is not None:
            init_fn(worker_id)
    except Exception as e:  # noqa: BLE001
        result_q.put((-1, _WorkerError(worker_id, e)))
        return
    while True:
        item = index_q.get()
        if item is None:
            break
        bi, idx = item
        try:
            out = collate_fn([dataset[i] for i in idx])
        except Exception as e:  # noqa: BLE001
            out = _WorkerError(worker_id, e)
        result_q.put((bi, out))


class _MultiProcessIter:
    """One epoch over worker processes: index lists round-robin out, results re-ordered in."""

    _POLL_S = 1.0

    def __init__(self, loader: DataLoader):
        import torch.multiprocessing as tmp

        self.loader = loader
        ctx = loader.multiprocessing_context
        if ctx is None or isinstance(ctx, str):
            ctx = tmp.get_context(ctx or "fork")
        W = loader.num_workers
        base_seed = int(torch.empty((), dtype=torch.int64).random_(generator=loader.generator).item())
        self.index_qs = [ctx.Queue() for _ in range(W)]
        self.result_q = ctx.Queue()
        self.workers = []
        for wid in range(W):
            w = ctx.Process(target=_worker_loop, args=(loader.dataset, loader.collate_fn, self.index_qs[wid],
                                                       self.result_q, base_seed, wid, W, loader.worker_init_fn),
                            daemon=True)
            w.start()
            self.workers.append(w)
        # pin-memory thread: result queue -> (pinned) local queue
        self.ready: "queue.Queue" = queue.Queue()
        self.stop = threading.Event()
        self.pin_thread = threading.Thread(target=self._pin_loop, daemon=True, name="ringdp-pin-memory")
        self.pin_thread.start()
        self.batches = loader._batches()
        self.sent = 0
        self.next = 0
        self.buf = {}
        self.done = False
        for _ in range(loader.prefetch_factor * W):
            self._put()

    def _pin_loop(self):
        while not self.stop.is_set():
            try:
                bi, data = self.result_q.get(timeout=0.1)
            except queue.Empty:
                continue
            except (EOFError, OSError):
                break
            if not isinstance(data, _WorkerError):
                try:
                    data = self.loader._pin(data)
                except Exception as e:  # noqa: BLE001
                    data = _WorkerError(-1, e)
            self.ready.put((bi, data))

    def _put(self):
        try:
            idx = next(self.batches)
        except StopIteration:
            return
        self.index_qs[self.sent % len(self.workers)].put((self.sent, idx))
        self.sent += 1

    def _shutdown(self):
        if self.done:
            return
        self.done = True
        for q in self.index_qs:
            try:
                q.put(None)
            except Exception:  # noqa: BLE001
                pass
        for w in self.workers:
            w.join(timeout=5)
            if w.is_alive():
                w.terminate()
        self.stop.set()
        self.pin_thread.join(timeout=5)

    def __iter__(self):
        return self

    def __next__(self):
        if self.next >= self.sent:
            self._shutdown()
            raise StopIteration
        waited = 0.0
        while self.next not in self.buf:
            try:
                bi, data = self.ready.get(timeout=self._POLL_S)
            except queue.Empty:
                waited += self._POLL_S
                dead = [w for w in self.workers if not w.is_alive()]
                if dead:
                    self._shutdown()
                    raise RuntimeError(f"DataLoader worker (pid(s) {', '.join(str(w.pid) for w in dead)}) "
                                       f"exited unexpectedly (exit code {dead[0].exitcode})")
                if self.loader.timeout and waited >= self.loader.timeout:
                    self._shutdown()
                    raise RuntimeError(f"DataLoader timed out after {self.loader.timeout} seconds")
                continue
            if isinstance(data, _WorkerError):
                self._shutdown()
                raise data.exc_type(data.msg) if data.exc_type is not KeyError else KeyError(data.msg)
            self.buf[bi] = data
        data = self.buf.pop(self.next)
        self.next += 1
        self._put()
        return data

    def __del__(self):
        try:
            self._shutdown()
        except Exception:  # noqa: BLE001
            pass


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
