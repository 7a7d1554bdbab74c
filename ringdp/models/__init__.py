"""ringdp.models - the reference's model families, MI355X-native."""
from .convnet import ConvNet  # noqa: F401

__all__ = ["ConvNet"]
