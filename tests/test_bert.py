"""The MI355X BERT encoder (models/bert.py) against ``transformers.BertForQuestionAnswering``:
same weights (via ``load_hf_state_dict``) -> same logits, loss and gradients (fp32, CPU path =
the composite reference of the fused ops).  The GPU kernels are pinned to the same composite in
tests/test_transformer_gpu.py."""
import pytest
import torch

from determined_1_amd.models.bert import BertEncoderConfig, BertForQA, load_hf_state_dict

transformers = pytest.importorskip("transformers")


def _pair(dropout=0.0):
    cfg = dict(vocab_size=1000, hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=128,
               hidden_dropout_prob=dropout, attention_probs_dropout_prob=dropout)
    torch.manual_seed(0)
    hf = transformers.BertForQuestionAnswering(transformers.BertConfig(**cfg, attn_implementation="sdpa"))
    ours = BertForQA(BertEncoderConfig(**cfg))
    load_hf_state_dict(ours, hf.state_dict())
    return hf, ours


def _batch(B=3, S=32):
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(1, 1000, (B, S), generator=g)
    tt = torch.zeros(B, S, dtype=torch.long)
    tt[:, S // 2:] = 1
    am = torch.ones(B, S, dtype=torch.long)
    am[0, -5:] = 0  # one padded example exercises the additive mask
    s = torch.randint(0, S, (B,), generator=g)
    e = torch.clamp(s + 3, max=S - 1)
    return ids, tt, am, s, e


def test_forward_matches_hf():
    hf, ours = _pair()
    hf.eval()
    ours.eval()
    ids, tt, am, s, e = _batch()
    a = hf(input_ids=ids, token_type_ids=tt, attention_mask=am, start_positions=s, end_positions=e)
    b = ours(input_ids=ids, token_type_ids=tt, attention_mask=am, start_positions=s, end_positions=e)
    torch.testing.assert_close(b.start_logits, a.start_logits, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(b.end_logits, a.end_logits, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(b.loss, a.loss, atol=1e-5, rtol=1e-5)


def test_gradients_match_hf():
    hf, ours = _pair()
    hf.train()
    ours.train()
    ids, tt, am, s, e = _batch()
    hf(input_ids=ids, token_type_ids=tt, attention_mask=am, start_positions=s, end_positions=e).loss.backward()
    ours(input_ids=ids, token_type_ids=tt, attention_mask=am, start_positions=s, end_positions=e).loss.backward()
    hg = {k: v.grad for k, v in hf.named_parameters()}
    og = dict(ours.named_parameters())
    pre = "bert.encoder.layer.1."
    q = torch.cat([hg[pre + f"attention.self.{m}.weight"] for m in ("query", "key", "value")])
    torch.testing.assert_close(og["layers.1.qkv.weight"].grad, q, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(og["layers.0.ffn_ln.weight"].grad, hg["bert.encoder.layer.0.output.LayerNorm.weight"],
                               atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(og["layers.0.ffn_in.bias"].grad, hg["bert.encoder.layer.0.intermediate.dense.bias"],
                               atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(og["embeddings.word_embeddings.weight"].grad,
                               hg["bert.embeddings.word_embeddings.weight"], atol=1e-5, rtol=1e-4)


def test_param_count_matches_bert_base():
    m = BertForQA(BertEncoderConfig())
    assert sum(p.numel() for p in m.parameters()) == 108893186  # bert-base-uncased + QA head


def test_sequence_classification_matches_hf():
    """models/bert_glue.py BertForSequenceClassification vs transformers (pooler + classifier)."""
    from determined_1_amd.models.bert_glue import BertForSequenceClassification
    from determined_1_amd.models.bert_glue import load_hf_state_dict as load_cls

    cfg = dict(vocab_size=1000, hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=128,
               hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    torch.manual_seed(0)
    hf = transformers.BertForSequenceClassification(transformers.BertConfig(**cfg, num_labels=2,
                                                                            attn_implementation="sdpa"))
    ours = BertForSequenceClassification(BertEncoderConfig(**cfg), num_labels=2)
    load_cls(ours, hf.state_dict())
    ids, tt, am, _, _ = _batch()
    labels = torch.tensor([0, 1, 1])
    a = hf(input_ids=ids, token_type_ids=tt, attention_mask=am, labels=labels)
    b = ours(input_ids=ids, token_type_ids=tt, attention_mask=am, labels=labels)
    torch.testing.assert_close(b.logits, a.logits, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(b.loss, a.loss, atol=1e-5, rtol=1e-5)
    a.loss.backward()
    b.loss.backward()
    torch.testing.assert_close(ours.pooler.weight.grad, hf.bert.pooler.dense.weight.grad, atol=1e-5, rtol=1e-4)
