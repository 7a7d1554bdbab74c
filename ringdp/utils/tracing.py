"""roctx ranges for rocprofv3 (``--marker-trace``): ``RINGDP_ROCTX=1`` or ``enable()`` turns them on.

SURVEY.md §5 "Tracing / profiling": the reference has none; upstream wraps DDP forward in
``record_function("DistributedDataParallel.forward")``.  ringdp emits roctx ranges around DDP forward
/ backward, the optimizer step and bench phases, plus a marker per bucket launch from the C++ reducer,
so a ``rocprofv3 --kernel-trace --marker-trace`` timeline shows which kernels and RCCL calls belong to
which phase.  Disabled ranges cost one attribute lookup.

    with ringdp.utils.tracing.range("my-phase"):
        ...
"""
from __future__ import annotations

import contextlib
import functools

from .._native import C


def enable(on: bool = True) -> None:
    C.trace_set_enabled(bool(on))


def enabled() -> bool:
    return bool(C.trace_enabled())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx/roctx naming
    on = C.trace_enabled()
    if on:
        C.trace_push(name)
    try:
        yield
    finally:
        if on:
            C.trace_pop()


def mark(msg: str) -> None:
    if C.trace_enabled():
        C.trace_mark(msg)


def annotate(name: str):
    """Decorator form of :func:`range`."""

    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*a, **kw):
            with range(name):
                return fn(*a, **kw)

        return wrapper

    return deco
