"""BERT-base SQuAD fine-tuning trial (reference examples/nlp/bert_squad_pytorch): see
determined_1_amd/models/bert.py."""
from determined_1_amd.models.bert import BertSQuADTrial as BertSQuADPyTorch  # noqa: F401
