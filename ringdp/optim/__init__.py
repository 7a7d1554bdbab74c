"""ringdp.optim - optimizers with fused CDNA4 update kernels."""
from .sgd import SGD  # noqa: F401

__all__ = ["SGD"]
