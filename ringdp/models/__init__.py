"""ringdp.models - the reference's model families, MI355X-native."""
from .convnet import ConvNet  # noqa: F401
from .resnet import ResNet, resnet18, resnet34, resnet50  # noqa: F401
from .vit import VisionTransformer, vit_b_16, vit_tiny  # noqa: F401

__all__ = ["ConvNet", "ResNet", "resnet18", "resnet34", "resnet50", "VisionTransformer", "vit_b_16", "vit_tiny"]
