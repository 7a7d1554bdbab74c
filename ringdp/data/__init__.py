"""ringdp.data - samplers, datasets, transforms and on-device loaders."""
from .sampler import DeviceDistributedSampler, DistributedSampler  # noqa: F401

__all__ = ["DistributedSampler", "DeviceDistributedSampler"]
