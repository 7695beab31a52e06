"""The ALBERT QA model (models/albert.py: factorised embeddings + one shared fused encoder layer,
tanh GELU) against ``transformers.AlbertForQuestionAnswering``: same weights -> same logits, loss
and gradients on the CPU composite path.  The GPU kernels (H = 4096 LayerNorm, tanh GELU) are
pinned to the same composite in tests/test_transformer_gpu.py."""
import pytest
import torch

from determined_1_amd.models.albert import XXLARGE_V2, AlbertConfig, AlbertForQA, load_hf_state_dict

transformers = pytest.importorskip("transformers")

CFG = dict(vocab_size=1000, embedding_size=16, hidden_size=64, num_hidden_layers=3, num_attention_heads=4,
           intermediate_size=128, hidden_act="gelu_new", hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)


def _pair():
    torch.manual_seed(0)
    hf = transformers.AlbertForQuestionAnswering(transformers.AlbertConfig(**CFG, attn_implementation="eager"))
    ours = AlbertForQA(AlbertConfig(**CFG))
    load_hf_state_dict(ours, hf.state_dict())
    return hf, ours


def _batch(B=3, S=32):
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(1, 1000, (B, S), generator=g)
    tt = torch.zeros(B, S, dtype=torch.long)
    tt[:, S // 2:] = 1
    am = torch.ones(B, S, dtype=torch.long)
    am[0, -5:] = 0
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


def test_shared_layer_gradients_match_hf():
    hf, ours = _pair()
    ids, tt, am, s, e = _batch()
    hf(input_ids=ids, token_type_ids=tt, attention_mask=am, start_positions=s, end_positions=e).loss.backward()
    ours(input_ids=ids, token_type_ids=tt, attention_mask=am, start_positions=s, end_positions=e).loss.backward()
    hg = {k: v.grad for k, v in hf.named_parameters()}
    og = dict(ours.named_parameters())
    pre = "albert.encoder.albert_layer_groups.0.albert_layers.0."
    q = torch.cat([hg[pre + f"attention.{m}.weight"] for m in ("query", "key", "value")])
    torch.testing.assert_close(og["layer.qkv.weight"].grad, q, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(og["layer.ffn_in.bias"].grad, hg[pre + "ffn.bias"], atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(og["layer.ffn_ln.weight"].grad, hg[pre + "full_layer_layer_norm.weight"],
                               atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(og["embedding_hidden_mapping_in.weight"].grad,
                               hg["albert.encoder.embedding_hidden_mapping_in.weight"], atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(og["embeddings.word_embeddings.weight"].grad,
                               hg["albert.embeddings.word_embeddings.weight"], atol=1e-5, rtol=1e-4)


def test_xxlarge_v2_param_count():
    # albert-xxlarge-v2: 222.6M encoder+embedding parameters (+ 8194 for the QA head)
    with torch.device("meta"):
        m = AlbertForQA(AlbertConfig(**XXLARGE_V2))
    hf_cfg = transformers.AlbertConfig(**XXLARGE_V2)
    with torch.device("meta"):
        hf = transformers.AlbertForQuestionAnswering(hf_cfg)
    assert sum(p.numel() for p in m.parameters()) == sum(p.numel() for p in hf.parameters())


def test_shared_weight_grads_accumulate_through_gemm():
    """SharedWeightGrads: 3 uses of one weight -> the last backward use returns the summed dW
    (GEMM beta=1 accumulation), the others None; equals autograd's own summation."""
    from determined_1_amd.ops import transformer as tfops

    torch.manual_seed(0)
    w = torch.randn(16, 16, requires_grad=True)
    x = torch.randn(5, 16, requires_grad=True)
    acc = tfops.SharedWeightGrads()
    y = x
    for _ in range(3):
        y = torch.tanh(tfops._Linear.apply(y, w, None, tfops._track(acc, w)))
    y.sum().backward()
    g_acc, gx_acc = w.grad.clone(), x.grad.clone()
    w.grad = None
    x.grad = None
    y = x
    for _ in range(3):
        y = torch.tanh(torch.nn.functional.linear(y, w))
    y.sum().backward()
    torch.testing.assert_close(g_acc, w.grad)
    torch.testing.assert_close(gx_acc, x.grad)
    assert not any(st[1] is not None for st in acc._state.values())
