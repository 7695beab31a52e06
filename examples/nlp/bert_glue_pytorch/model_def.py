"""BERT GLUE (MRPC) fine-tuning trial (reference examples/nlp/bert_glue_pytorch): see
determined_1_amd/models/bert_glue.py.  Synthetic MRPC-shaped sentence pairs (no network here)."""
from determined_1_amd.models.bert_glue import BertGLUETrial as BertPytorch  # noqa: F401
