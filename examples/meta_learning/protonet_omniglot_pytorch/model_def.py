"""Prototypical-network few-shot trial (reference examples/meta_learning/protonet_omniglot_pytorch):
see determined_1_amd/models/protonet.py.  Synthetic glyph episodes stand in for Omniglot."""
from determined_1_amd.models.protonet import ProtoNetTrial as OmniglotProtoNetTrial  # noqa: F401
