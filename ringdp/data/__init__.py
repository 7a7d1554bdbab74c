"""ringdp.data - samplers, datasets, transforms and loaders (host and HBM-resident)."""
from . import transforms  # noqa: F401
from .datasets import (  # noqa: F401
    CIFAR10,
    MNIST,
    ImageDataset,
    SyntheticImages,
    cifar10_or_synthetic,
    mnist_or_synthetic,
)
from .loader import DataLoader, DeviceLoader, RandomSampler, SequentialSampler  # noqa: F401
from .sampler import DeviceDistributedSampler, DistributedSampler  # noqa: F401

__all__ = [
    "DistributedSampler", "DeviceDistributedSampler", "DataLoader", "DeviceLoader", "RandomSampler",
    "SequentialSampler", "MNIST", "CIFAR10", "SyntheticImages", "ImageDataset", "mnist_or_synthetic",
    "cifar10_or_synthetic", "transforms",
]
