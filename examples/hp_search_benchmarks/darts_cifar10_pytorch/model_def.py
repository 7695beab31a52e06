"""DARTS CIFAR-10 architecture search as hyperparameter search (reference
examples/hp_search_benchmarks/darts_cifar10_pytorch): see determined_1_amd/models/darts.py."""
from determined_1_amd.models.darts import DARTSCNNTrial  # noqa: F401
