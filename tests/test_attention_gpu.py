"""det_attention.hip (MFMA flash attention) vs an fp64 composite on the CPU: bf16 head_dim
32/64/128 and fp32 32/64, tail blocks (any Lq/Lk), cross-attention, per-key and full additive /
boolean masks with broadcast strides, the kernels' own dropout masks, and zero-fallback checks at
the BERT, ALBERT and DETR encoder shapes."""
import pytest
import torch

from determined_1_amd.ops import transformer as tfops

pytestmark = pytest.mark.gpu


def _ref_attention(q, k, v, nh, bias, keep=None, keep_scale=1.0):
    """fp64 softmax(q k^T * d^-1/2 + bias) [o keep] v on [B, L, H] tensors."""
    B, Lq, H = q.shape
    hd = H // nh

    def heads(t):
        return t.reshape(B, t.shape[1], nh, hd).transpose(1, 2)

    s = heads(q) @ heads(k).transpose(-1, -2) * hd ** -0.5
    if bias is not None:
        s = s + bias
    pr = torch.softmax(s, dim=-1)
    if keep is not None:
        pr = pr * keep.to(pr.dtype) * keep_scale
    return (pr @ heads(v)).transpose(1, 2).reshape(B, Lq, H)


def _bias(kind, B, nh, Lq, Lk, g):
    if kind is None:
        return None, None
    if kind == "key":  # [B, 1, 1, Lk] padding mask, additive
        am = torch.ones(B, Lk)
        am[-1, Lk - max(1, Lk // 5):] = 0
        b = (1.0 - am)[:, None, None, :] * -10000.0
        return b, b
    if kind == "full_b":  # [B, 1, Lq, Lk] additive
        b = torch.randn(B, 1, Lq, Lk, generator=g, dtype=torch.float64)
        return b, b
    if kind == "full_h":  # [1, nh, Lq, Lk] additive (per-head bias, broadcast over the batch)
        b = torch.randn(1, nh, Lq, Lk, generator=g, dtype=torch.float64) * 2
        return b, b
    if kind == "causal":  # boolean keep-mask [Lq, Lk] (SDPA semantics)
        m = torch.ones(Lq, Lk, dtype=torch.bool).tril(diagonal=Lk - Lq)
        return m, torch.zeros(Lq, Lk, dtype=torch.float64).masked_fill(~m, float("-inf"))
    raise ValueError(kind)


CASES = [
    # dtype, hd, B, nh, Lq, Lk, mask, packed
    (torch.bfloat16, 64, 4, 12, 384, 384, "key", True),  # BERT-base SQuAD
    (torch.bfloat16, 64, 2, 4, 200, 200, "key", True),  # tail blocks
    (torch.bfloat16, 128, 2, 4, 333, 333, "full_b", True),  # head_dim 128, [B,1,S,S] mask
    (torch.bfloat16, 32, 2, 8, 100, 850, "key", False),  # DETR cross-attention shape
    (torch.bfloat16, 64, 2, 2, 130, 130, "causal", True),
    (torch.float32, 32, 2, 8, 850, 850, "key", False),  # DETR encoder, fp32 reference precision
    (torch.float32, 32, 2, 8, 100, 100, None, False),  # DETR decoder self-attention
    (torch.float32, 64, 2, 4, 512, 512, "key", True),  # ALBERT fp32 reference config shape
    (torch.float32, 64, 2, 3, 77, 130, "full_h", False),
    (torch.bfloat16, 128, 1, 2, 1000, 64, None, False),
]


@pytest.mark.parametrize("dt,hd,B,nh,Lq,Lk,mask,packed", CASES)
def test_attention_matches_fp64(gpu, dt, hd, B, nh, Lq, Lk, mask, packed):
    g = torch.Generator().manual_seed(hd + Lq + Lk)
    H = nh * hd
    assert tfops.mfma_attention_supported(Lq, hd, dt, Lk)
    if packed:
        assert Lq == Lk
        x = (torch.randn(B, Lq, 3 * H, generator=g, dtype=torch.float64) * 1.5).to(dt)
        ins = [x[..., :H], x[..., H:2 * H], x[..., 2 * H:]]
    else:
        ins = [(torch.randn(B, L, H, generator=g, dtype=torch.float64) * 1.5).to(dt) for L in (Lq, Lk, Lk)]
    dy = torch.randn(B, Lq, H, generator=g, dtype=torch.float64).to(dt)
    dev_mask, ref_mask = _bias(mask, B, nh, Lq, Lk, g)
    ref_ins = [t.double().clone().requires_grad_(True) for t in ins]
    ref = _ref_attention(*ref_ins, nh, ref_mask)
    ref.backward(dy.double())

    before = tfops.FALLBACKS["count"]
    m = None
    if dev_mask is not None:
        m = dev_mask.to(gpu) if dev_mask.dtype == torch.bool else dev_mask.to(gpu, dt)
    if packed:
        x_d = x.to(gpu).requires_grad_(True)
        out = tfops.qkv_self_attention(x_d, nh, m, 0.0)
        out.backward(dy.to(gpu))
        grads = [x_d.grad[..., :H], x_d.grad[..., H:2 * H], x_d.grad[..., 2 * H:]]
    else:
        d_ins = [t.to(gpu).requires_grad_(True) for t in ins]
        out = tfops.attention(*d_ins, nh, attn_bias=m)
        out.backward(dy.to(gpu))
        grads = [t.grad for t in d_ins]
    assert tfops.FALLBACKS["count"] == before, "attention fell back to the composite path"
    tol = 2e-2 if dt == torch.bfloat16 else 2e-4
    for name, got, want in (("out", out, ref), ("dq", grads[0], ref_ins[0].grad), ("dk", grads[1], ref_ins[1].grad),
                            ("dv", grads[2], ref_ins[2].grad)):
        got = got.detach().double().cpu()
        want = want.detach()
        assert torch.isfinite(got).all(), name
        err = (got - want).abs().max().item() / max(want.abs().max().item(), 1e-12)
        assert err < tol, (name, err)


@pytest.mark.parametrize("dt,hd,B,nh,Lq,Lk,p", [
    (torch.bfloat16, 64, 3, 2, 256, 256, 0.1),
    (torch.bfloat16, 64, 1, 2, 512, 512, 0.2),
    (torch.bfloat16, 64, 2, 3, 130, 130, 0.1),  # Lk not a multiple of 4 or 64
    (torch.float32, 32, 2, 2, 90, 203, 0.1),  # cross-attention, odd key count
    (torch.bfloat16, 128, 1, 2, 192, 192, 0.1),
])
def test_attention_dropout(gpu, monkeypatch, dt, hd, B, nh, Lq, Lk, p):
    """fwd + bwd with dropout vs the fp64 composite using the kernels' own keep mask."""
    g = torch.Generator().manual_seed(7)
    H = nh * hd
    ins = [torch.randn(B, L, H, generator=g, dtype=torch.float64).to(dt) for L in (Lq, Lk, Lk)]
    dy = torch.randn(B, Lq, H, generator=g, dtype=torch.float64).to(dt)
    am = torch.ones(B, Lk)
    am[-1, Lk - 19:] = 0
    bias = (1.0 - am)[:, None, None, :] * -10000.0
    seed, off = 4242, 9
    monkeypatch.setattr(tfops, "next_rng", lambda: (seed, off))
    keep = tfops.attention_dropout_mask(B, nh, Lq, p, seed, off, torch.device(gpu), Lk=Lk).cpu()
    thr = min(65535, int(p * 65536 + 0.5))
    assert abs(keep.float().mean().item() - (1 - thr / 65536)) < 1e-2
    ref_ins = [t.double().clone().requires_grad_(True) for t in ins]
    ref = _ref_attention(*ref_ins, nh, bias.double(), keep, 65536.0 / (65536 - thr))
    ref.backward(dy.double())
    d_ins = [t.to(gpu).requires_grad_(True) for t in ins]
    out = tfops.attention(*d_ins, nh, attn_bias=bias.to(gpu, dt), p=p, training=True)
    out.backward(dy.to(gpu))
    tol = 3e-2 if dt == torch.bfloat16 else 2e-4
    for name, got, want in (("out", out, ref),) + tuple((f"d{i}", a.grad, r.grad) for i, a, r in zip("qkv", d_ins, ref_ins)):
        got, want = got.detach().double().cpu(), want.detach()
        err = (got - want).abs().max().item() / max(want.abs().max().item(), 1e-12)
        assert err < tol, (name, err)


def test_zero_attention_fallbacks_at_model_shapes(gpu):
    """BERT-base (bf16 autocast, S 384), ALBERT (fp32 reference precision, head_dim 64) and the DETR
    transformer (fp32, head_dim 32, S = 25x34 feature pixels, 100 queries): fwd + bwd never leave
    det_attention.hip."""
    from determined_1_amd.models.albert import AlbertConfig, AlbertForQA
    from determined_1_amd.models.bert import BertEncoderConfig, BertForQA
    from determined_1_amd.models.detr import Transformer

    torch.manual_seed(0)
    before = tfops.FALLBACKS["count"]
    bert = BertForQA(BertEncoderConfig(vocab_size=1024, hidden_size=768, num_hidden_layers=1, num_attention_heads=12,
                                       intermediate_size=3072)).to(gpu)
    ids = torch.randint(1, 1024, (2, 384), device=gpu)
    am = torch.ones_like(ids)
    am[1, -50:] = 0
    s = torch.randint(0, 384, (2,), device=gpu)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = bert(ids, None, am, s, s)
    out.loss.backward()
    albert = AlbertForQA(AlbertConfig(vocab_size=1024, embedding_size=128, hidden_size=512, num_hidden_layers=2,
                                      num_attention_heads=8, intermediate_size=1024)).to(gpu)
    out = albert(ids, None, am, s, s)
    out.loss.backward()
    tr = Transformer(d=256, heads=8, enc_layers=1, dec_layers=1).to(gpu)
    src = torch.randn(2, 850, 256, device=gpu)
    pos = torch.randn(2, 850, 256, device=gpu)
    mask = torch.zeros(2, 850, dtype=torch.bool, device=gpu)
    mask[1, 800:] = True
    hs = tr(src, mask, torch.randn(100, 256, device=gpu), pos)
    hs.float().pow(2).mean().backward()
    assert tfops.FALLBACKS["count"] == before
    torch.cuda.synchronize()


@pytest.mark.parametrize("dt,hd,B,nh,Lq,Lk,mask", [
    (torch.bfloat16, 64, 4, 12, 384, 384, "key"),     # BERT-base SQuAD
    (torch.bfloat16, 128, 2, 4, 333, 200, "full_b"),  # cross-attention, full bias, tails
    (torch.float32, 32, 2, 8, 100, 850, None),        # DETR decoder cross-attention
])
def test_merged_backward_equals_two_launch_backward(gpu, dt, hd, B, nh, Lq, Lk, mask):
    """The merged backward (D pre-pass, then dQ and dK/dV work in one grid) computes exactly what the
    dQ-then-dK/dV launches do: the same D (same summation order) and the same per-tile work."""
    from determined_1_amd.ops import _lib

    lib = _lib.get_lib()
    g = torch.Generator().manual_seed(7)
    H = nh * hd
    ins = [(torch.randn(B, L, H, generator=g) * 1.5).to(dt) for L in (Lq, Lk, Lk)]
    dy = torch.randn(B, Lq, H, generator=g).to(dt)
    dev_mask, _ = _bias(mask, B, nh, Lq, Lk, g)
    m = None if dev_mask is None else dev_mask.to(gpu, dt)
    res = {}
    try:
        for merged in (0, 1):
            lib.det_attn_set_bwd_merged(merged)
            d_ins = [t.to(gpu).requires_grad_(True) for t in ins]
            out = tfops.attention(*d_ins, nh, attn_bias=m)
            out.backward(dy.to(gpu))
            res[merged] = [out.detach().clone()] + [t.grad.clone() for t in d_ins]
    finally:
        lib.det_attn_set_bwd_merged(-2)
    for name, a, b in zip(("out", "dq", "dk", "dv"), res[0], res[1]):
        assert torch.equal(a, b), name
