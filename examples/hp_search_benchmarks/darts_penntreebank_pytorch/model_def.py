"""DARTS recurrent-cell search on Penn Treebank as hyperparameter search (reference
examples/hp_search_benchmarks/darts_penntreebank_pytorch): see determined_1_amd/models/darts_rnn.py."""
from determined_1_amd.models.darts_rnn import DARTSRNNTrial  # noqa: F401
