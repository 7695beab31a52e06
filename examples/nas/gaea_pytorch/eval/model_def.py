"""GAEA searched-cell ImageNet evaluation (reference examples/nas/gaea_pytorch/eval):
see determined_1_amd/models/gaea.py."""
from determined_1_amd.models.gaea import GAEAEvalTrial  # noqa: F401
