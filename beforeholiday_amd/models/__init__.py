"""Reference workloads built from this library's layers."""
from .resnet import ResNet, Bottleneck, resnet50, resnet18_like, resnet50_fused

__all__ = ["ResNet", "Bottleneck", "resnet50", "resnet18_like", "resnet50_fused"]
