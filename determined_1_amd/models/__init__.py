"""Model zoo used by the examples, tests and ``bench.py`` (torchvision is not available on the
image, so the reference's vision models are written out here)."""
from determined_1_amd.models.resnet import ResNet, resnet18, resnet34, resnet50, resnet101, resnet152
from determined_1_amd.models.small import CIFAR10CNN, MNISTNet, OneVarModel, XORNet

__all__ = [
    "CIFAR10CNN",
    "MNISTNet",
    "OneVarModel",
    "ResNet",
    "XORNet",
    "resnet18",
    "resnet34",
    "resnet50",
    "resnet101",
    "resnet152",
]
