"""ALBERT-xxlarge-v2 SQuAD 2.0 fine-tuning trial (reference examples/nlp/albert_squad_pytorch):
see determined_1_amd/models/albert.py.  Synthetic SQuAD-shaped features (no network here)."""
from determined_1_amd.models.albert import AlbertSQuADTrial as AlbertSQuADPyTorch  # noqa: F401
