"""GAEA weight-sharing architecture search (reference examples/nas/gaea_pytorch/search):
see determined_1_amd/models/gaea.py."""
from determined_1_amd.models.gaea import GAEASearchTrial  # noqa: F401
