"""ResNet-50 ImageNet-shape trial: the north-star benchmark (bench.py runs the same class)."""
from determined_1_amd.models.imagenet_trial import ResNetImageNetTrial  # noqa: F401
