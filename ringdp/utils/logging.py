"""Rank-aware logging in the reference scripts' formats.

``ref/launch_dist.py:93-102``: ``Epoch [e/E], Step [i/N], Loss: x.xxxx`` every 100 steps and
``Training complete in: <timedelta>``; ``ref/example_mp.py:115-127``: running loss + top-1 accuracy
every 25 steps on global rank 0.  Printing is gated on the GLOBAL rank by default (the reference
gates on local rank, i.e. once per node - ``rank_filter="local"`` keeps that behaviour).
"""
from __future__ import annotations

import os
import sys
import time
from datetime import datetime, timedelta


def _ranks():
    r = int(os.environ.get("RANK", "0") or 0)
    lr = int(os.environ.get("LOCAL_RANK", str(r)) or 0)
    try:
        from .. import distributed as dist

        if dist.is_initialized():
            r = dist.get_rank()
    except Exception:  # pragma: no cover - logging must never fail
        pass
    return r, lr


def is_log_rank(rank_filter: str = "global") -> bool:
    r, lr = _ranks()
    return (lr if rank_filter == "local" else r) == 0


def log(*args, rank_filter: str = "global", **kw) -> None:
    if is_log_rank(rank_filter):
        print(*args, **kw)
        sys.stdout.flush()


def step_line(epoch: int, epochs: int, step: int, total: int, loss: float) -> str:
    return "Epoch [{}/{}], Step [{}/{}], Loss: {:.4f}".format(epoch + 1, epochs, step + 1, total, loss)


class Meter:
    """Running mean of loss and top-1 accuracy (example_mp.py-style metrics)."""

    def __init__(self):
        self.loss_sum = 0.0
        self.correct = 0
        self.count = 0
        self.steps = 0

    def update(self, loss: float, correct: int, n: int) -> None:
        self.loss_sum += loss
        self.correct += correct
        self.count += n
        self.steps += 1

    @property
    def loss(self) -> float:
        return self.loss_sum / max(1, self.steps)

    @property
    def acc(self) -> float:
        return 100.0 * self.correct / max(1, self.count)


class WallClock:
    def __init__(self):
        self.start = datetime.now()
        self.t0 = time.perf_counter()

    def elapsed(self) -> timedelta:
        return datetime.now() - self.start

    def seconds(self) -> float:
        return time.perf_counter() - self.t0
