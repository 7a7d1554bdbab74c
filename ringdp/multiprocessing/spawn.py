"""spawn(fn, args, nprocs) - one fresh interpreter per rank with failure propagation.

Parity: ``torch/multiprocessing/spawn.py:79-340``, used by the reference at
``ref/mpspawn_dist.py:140`` and ``ref/example_mp.py:27``:

* children are started with the ``spawn`` start method and run ``fn(i, *args)``;
* each child gets PDEATHSIG=SIGINT so it dies with its parent;
* an uncaught exception in a child is written (as text) to a per-child error file and the child
  exits non-zero;
* the parent joins on process sentinels; on the first failure it SIGTERMs, then SIGKILLs the
  remaining children and raises ProcessRaisedException (with the child traceback) or
  ProcessExitedException (exit code / signal).
"""
from __future__ import annotations

import ctypes
import multiprocessing
import multiprocessing.connection
import os
import signal
import sys
import tempfile
import time
import traceback
from typing import Any, Callable, Optional, Tuple


class ProcessException(Exception):
    def __init__(self, msg: str, error_index: int, pid: int):
        super().__init__(msg)
        self.msg = msg
        self.error_index = error_index
        self.pid = pid

    def __reduce__(self):
        return type(self), (self.msg, self.error_index, self.pid)


class ProcessRaisedException(ProcessException):
    """A child process raised an exception."""


class ProcessExitedException(ProcessException):
    """A child process exited with a non-zero code or died from a signal."""

    def __init__(self, msg: str, error_index: int, error_pid: int, exit_code: int, signal_name: Optional[str] = None):
        super().__init__(msg, error_index, error_pid)
        self.exit_code = exit_code
        self.signal_name = signal_name

    def __reduce__(self):
        return type(self), (self.msg, self.error_index, self.pid, self.exit_code, self.signal_name)


def _set_pdeathsig(sig=signal.SIGINT):
    try:
        libc = ctypes.CDLL("libc.so.6", use_errno=True)
        PR_SET_PDEATHSIG = 1
        libc.prctl(PR_SET_PDEATHSIG, int(sig))
    except OSError:
        pass


def _wrap(fn: Callable, i: int, args: Tuple, error_file: str):
    _set_pdeathsig(signal.SIGINT)
    try:
        fn(i, *args)
    except KeyboardInterrupt:
        pass
    except Exception:
        with open(error_file, "w") as f:
            f.write(traceback.format_exc())
        sys.exit(1)


class ProcessContext:
    def __init__(self, processes, error_files):
        self.error_files = error_files
        self.processes = processes
        self.sentinels = {p.sentinel: i for i, p in enumerate(processes)}

    def pids(self):
        return [int(p.pid) for p in self.processes]

    def _terminate_all(self, grace: float = 10.0):
        for p in self.processes:
            if p.is_alive():
                p.terminate()
        deadline = time.monotonic() + grace
        for p in self.processes:
            p.join(max(0.0, deadline - time.monotonic()))
        for p in self.processes:
            if p.is_alive():
                p.kill()
                p.join()

    def join(self, timeout: Optional[float] = None, grace_period: float = 10.0) -> bool:
        """True when every process exited cleanly; raises on the first failure."""
        if not self.sentinels:
            return True
        ready = multiprocessing.connection.wait(self.sentinels.keys(), timeout=timeout)
        error_index = None
        for s in ready:
            i = self.sentinels.pop(s)
            p = self.processes[i]
            p.join()
            if p.exitcode != 0:
                error_index = i
                break
        if error_index is None:
            return len(self.sentinels) == 0
        self._terminate_all(grace_period)
        failed = self.processes[error_index]
        err_file = self.error_files[error_index]
        tb = ""
        if os.path.exists(err_file) and os.path.getsize(err_file) > 0:
            with open(err_file) as f:
                tb = f.read()
        if tb:
            msg = f"\n\n-- Process {error_index} terminated with the following error:\n{tb}"
            raise ProcessRaisedException(msg, error_index, failed.pid)
        code = failed.exitcode
        if code < 0:
            name = signal.Signals(-code).name
            raise ProcessExitedException(f"process {error_index} terminated with signal {name}",
                                         error_index, failed.pid, code, name)
        raise ProcessExitedException(f"process {error_index} terminated with exit code {code}",
                                     error_index, failed.pid, code)


def start_processes(fn: Callable, args: Tuple = (), nprocs: int = 1, join: bool = True,
                    daemon: bool = False, start_method: str = "spawn"):
    ctx = multiprocessing.get_context(start_method)
    error_files = []
    processes = []
    for i in range(nprocs):
        fd, path = tempfile.mkstemp(prefix=f"ringdp_spawn_{i}_", suffix=".err")
        os.close(fd)
        os.unlink(path)
        error_files.append(path)
        p = ctx.Process(target=_wrap, args=(fn, i, args, path), daemon=daemon)
        p.start()
        processes.append(p)
    context = ProcessContext(processes, error_files)
    if not join:
        return context
    try:
        while not context.join():
            pass
    finally:
        for f in error_files:
            if os.path.exists(f):
                os.unlink(f)
    return None


def spawn(fn: Callable, args: Tuple = (), nprocs: int = 1, join: bool = True, daemon: bool = False,
          start_method: str = "spawn"):
    """Spawns ``nprocs`` processes running ``fn(i, *args)`` (i = local process index)."""
    return start_processes(fn, args, nprocs, join, daemon, start_method)
