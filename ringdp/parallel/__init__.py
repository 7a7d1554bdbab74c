"""ringdp.parallel - data parallelism (DDP over RCCL / the host ring)."""
from . import comm_hooks  # noqa: F401
from .ddp import DistributedDataParallel, GradBucket  # noqa: F401

DDP = DistributedDataParallel

__all__ = ["DistributedDataParallel", "DDP", "GradBucket", "comm_hooks"]
