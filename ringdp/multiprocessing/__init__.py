"""ringdp.multiprocessing - process spawning for one-process-per-GPU training."""
from .spawn import ProcessContext, ProcessExitedException, ProcessRaisedException, spawn, start_processes  # noqa: F401

__all__ = ["spawn", "start_processes", "ProcessContext", "ProcessRaisedException", "ProcessExitedException"]
