"""Fused transformer kernels (ops/csrc/det_transformer.hip) vs the fp32 PyTorch composite."""
import os
import pytest
import torch
import torch.nn.functional as F

from determined_1_amd.ops import transformer as tfops

pytestmark = pytest.mark.gpu


def _tol(dt):
    return dict(atol=2e-4, rtol=2e-4) if dt == torch.float32 else dict(atol=4e-2, rtol=4e-2)


def _leaf(t, dev=None, dt=None):
    t = t.detach()
    if dev is not None:
        t = t.to(dev, dt)
    return t.clone().requires_grad_(True)


@pytest.mark.parametrize("rows,K,H,dt,p", [
    (512, 768, 768, torch.float32, 0.0),
    (4608, 768, 768, torch.bfloat16, 0.0),
    (1000, 3072, 768, torch.bfloat16, 0.1),
    (300, 256, 1024, torch.float32, 0.1),
    (77, 64, 200, torch.float32, 0.25),  # H not a multiple of 256 (inactive lanes)
    (768, 512, 4096, torch.bfloat16, 0.0),  # ALBERT-xxlarge width: workgroup-per-row kernels
    (700, 256, 4096, torch.bfloat16, 0.1),  # ... with dropout, rows not a multiple of the bwd grid
    (200, 256, 3072, torch.float32, 0.1),   # wide, inactive threads
    (64, 128, 6144, torch.float32, 0.0),    # two 16-B vectors per thread
])
def test_linear_dropout_add_layernorm(gpu, monkeypatch, rows, K, H, dt, p):
    torch.manual_seed(0)
    x = torch.randn(rows, K).to(dt).float()
    w = (torch.randn(H, K) / K ** 0.5).to(dt).float()
    b = (torch.randn(H) * 0.1).to(dt).float()
    r = torch.randn(rows, H).to(dt).float()
    g = (1 + 0.1 * torch.randn(H)).to(dt).float()
    be = (0.1 * torch.randn(H)).to(dt).float()
    dy = torch.randn(rows, H).to(dt).float()
    seed, off = 1234, 77
    monkeypatch.setattr(tfops, "next_rng", lambda: (seed, off))
    keep = tfops.dropout_mask(rows * H, p, seed, off, torch.device(gpu)).view(rows, H).cpu() if p > 0 else None
    if keep is not None:
        frac = keep.float().mean().item()
        assert abs(frac - (1 - p)) < 0.01, frac
    # reference: fp32 composite with the kernel's mask
    ref = [_leaf(t) for t in (x, w, b, r, g, be)]
    h = F.linear(ref[0], ref[1], ref[2])
    if keep is not None:
        h = h * keep.float() / (1 - p)
    yr = F.layer_norm(h + ref[3], (H,), ref[4], ref[5], 1e-12)
    yr.backward(dy)
    dut = [_leaf(t, gpu, dt) for t in (x, w, b, r, g, be)]
    before = tfops.FALLBACKS["count"]
    yd = tfops.linear_dropout_add_layernorm(*dut, p=p, eps=1e-12, training=True)
    yd.backward(dy.to(gpu, dt))
    assert tfops.FALLBACKS["count"] == before, "fused path fell back"
    tol = _tol(dt)
    torch.testing.assert_close(yd.float().cpu(), yr.detach(), **tol)
    for a, e, name in zip(dut, ref, ("dx", "dW", "db", "dres", "dgamma", "dbeta")):
        scale = max(1.0, e.grad.abs().max().item())
        torch.testing.assert_close(a.grad.float().cpu() / scale, e.grad / scale, **tol, msg=name)


@pytest.mark.parametrize("rows,K,N,dt,approx", [(512, 768, 3072, torch.float32, "none"),
                                                (4608, 768, 3072, torch.bfloat16, "none"),
                                                (100, 64, 264, torch.float32, "none"),
                                                (512, 256, 1024, torch.float32, "tanh"),
                                                (1536, 512, 2048, torch.bfloat16, "tanh")])
def test_linear_gelu(gpu, rows, K, N, dt, approx):
    torch.manual_seed(1)
    x, w, b = torch.randn(rows, K).to(dt).float(), (torch.randn(N, K) / K ** 0.5).to(dt).float(), torch.randn(N).to(dt).float()
    da = torch.randn(rows, N).to(dt).float()
    ref = [_leaf(t) for t in (x, w, b)]
    F.gelu(F.linear(*ref), approximate=approx).backward(da)
    dut = [_leaf(t, gpu, dt) for t in (x, w, b)]
    before = tfops.FALLBACKS["count"]
    out = tfops.linear_gelu(*dut, approximate=approx)
    out.backward(da.to(gpu, dt))
    assert tfops.FALLBACKS["count"] == before, "fused path fell back"
    tol = _tol(dt)
    torch.testing.assert_close(out.float().cpu(), F.gelu(F.linear(x, w, b), approximate=approx), **tol)
    for a, e in zip(dut, ref):
        scale = max(1.0, e.grad.abs().max().item())
        torch.testing.assert_close(a.grad.float().cpu() / scale, e.grad / scale, **tol)


@pytest.mark.parametrize("rows,K,N,dt", [(4608, 768, 2304, torch.bfloat16), (333, 128, 72, torch.float32)])
def test_linear_bias_grad(gpu, rows, K, N, dt):
    torch.manual_seed(2)
    x, w, b = torch.randn(rows, K).to(dt).float(), torch.randn(N, K).to(dt).float(), torch.randn(N).to(dt).float()
    dy = torch.randn(rows, N).to(dt).float()
    ref = [_leaf(t) for t in (x, w, b)]
    F.linear(*ref).backward(dy)
    dut = [_leaf(t, gpu, dt) for t in (x, w, b)]
    tfops.linear(*dut).backward(dy.to(gpu, dt))
    tol = _tol(dt)
    scale = max(1.0, ref[2].grad.abs().max().item())
    torch.testing.assert_close(dut[2].grad.float().cpu() / scale, ref[2].grad / scale, **tol)


def test_layer_norm(gpu):
    torch.manual_seed(3)
    x = torch.randn(1536, 768) * 3 + 1
    g, b = 1 + 0.1 * torch.randn(768), 0.1 * torch.randn(768)
    dy = torch.randn(1536, 768)
    ref = [_leaf(t) for t in (x, g, b)]
    F.layer_norm(ref[0], (768,), ref[1], ref[2], 1e-12).backward(dy)
    dut = [_leaf(t, gpu, torch.float32) for t in (x, g, b)]
    tfops.layer_norm(*dut, eps=1e-12).backward(dy.to(gpu))
    for a, e in zip(dut, ref):
        torch.testing.assert_close(a.grad.cpu(), e.grad, atol=3e-4, rtol=3e-4)


def test_bert_layer_fused_matches_composite(gpu, monkeypatch):
    """Whole fp32 BERT model on the GPU: fused kernels vs the composite path, dropout off."""
    from determined_1_amd.models.bert import BertEncoderConfig, BertForQA

    cfg = BertEncoderConfig(vocab_size=512, hidden_size=256, num_hidden_layers=2, num_attention_heads=4,
                            intermediate_size=1024, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    torch.manual_seed(4)
    m = BertForQA(cfg).to(gpu)
    ids = torch.randint(1, 512, (4, 128), device=gpu)
    am = torch.ones_like(ids)
    am[1, -10:] = 0
    s = torch.randint(0, 128, (4,), device=gpu)
    e = (s + 2).clamp(max=127)

    def run():
        m.zero_grad(set_to_none=True)
        out = m(ids, None, am, s, e)
        out.loss.backward()
        return out.loss.detach(), {k: p.grad.detach().clone() for k, p in m.named_parameters()}

    before = tfops.FALLBACKS["count"]
    loss_f, g_f = run()
    assert tfops.FALLBACKS["count"] == before
    monkeypatch.setattr(tfops, "_native", lambda *a, **k: False)
    monkeypatch.setenv("DET_ATTN", "composite")
    loss_c, g_c = run()
    torch.testing.assert_close(loss_f, loss_c, atol=1e-5, rtol=1e-5)
    for k in g_c:
        torch.testing.assert_close(g_f[k], g_c[k], atol=1e-4, rtol=1e-3, msg=k)


def test_albert_fused_matches_composite(gpu, monkeypatch):
    """Shared-layer ALBERT (tanh GELU, factorised embeddings) in fp32 on the GPU: fused kernels vs
    the composite path."""
    from determined_1_amd.models.albert import AlbertConfig, AlbertForQA

    cfg = AlbertConfig(vocab_size=512, embedding_size=64, hidden_size=256, num_hidden_layers=3, num_attention_heads=4,
                       intermediate_size=1024, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    torch.manual_seed(5)
    m = AlbertForQA(cfg).to(gpu)
    ids = torch.randint(1, 512, (2, 128), device=gpu)
    am = torch.ones_like(ids)
    am[0, -7:] = 0
    s = torch.randint(0, 128, (2,), device=gpu)
    e = (s + 2).clamp(max=127)

    def run():
        m.zero_grad(set_to_none=True)
        out = m(ids, None, am, s, e)
        out.loss.backward()
        return out.loss.detach(), {k: p.grad.detach().clone() for k, p in m.named_parameters()}

    before = tfops.FALLBACKS["count"]
    loss_f, g_f = run()
    assert tfops.FALLBACKS["count"] == before
    monkeypatch.setattr(tfops, "_native", lambda *a, **k: False)
    monkeypatch.setenv("DET_ATTN", "composite")
    loss_c, g_c = run()
    torch.testing.assert_close(loss_f, loss_c, atol=1e-5, rtol=1e-5)
    for k in g_c:
        torch.testing.assert_close(g_f[k], g_c[k], atol=1e-4, rtol=1e-3, msg=k)


def test_bert_trial_direct_gradient_landing(gpu, monkeypatch):
    """BERT trial on the GPU through the real controller (arenas, GradSink, fused AdamW): dW GEMMs
    writing straight into the gradient arena (ops.arena.landing_buffer) give the same parameters
    after 3 steps as the copy-landing path, and the landing copy really is skipped for them."""
    import copy as _copy

    from determined_1_amd.experimental import load_model_def

    BertSQuADTrial = load_model_def(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "nlp", "bert_squad_pytorch")).BertSQuADTrial
    from determined_1_amd.ops import arena
    from tests.utils import Recorder, run

    hp = {"global_batch_size": 4, "num_hidden_layers": 2, "hidden_size": 128, "num_attention_heads": 2,
          "intermediate_size": 512, "max_seq_length": 128, "amp": "O2", "train_records": 64, "validation_records": 8,
          "learning_rate": 1e-3}
    out = {}

    for direct in (False, True):
        monkeypatch.setattr(arena, "DIRECT_LANDING", direct)
        tfops.reset_rng()  # same dropout masks in both runs (the trial seeding resets the stream too)
        landed = []
        orig = arena.landing_buffer

        def spy(p, _orig=orig, _landed=landed):
            b = _orig(p)
            if b is not None:
                _landed.append(b.data_ptr())
            return b

        monkeypatch.setattr(arena, "landing_buffer", spy)
        monkeypatch.setattr(tfops, "landing_buffer", spy)
        ctrl, _ = run(BertSQuADTrial, _copy.deepcopy(hp), Recorder().train(1, 3, 0), trial_seed=3, use_gpu=True)
        out[direct] = (torch.cat([p.detach().float().reshape(-1) for p in ctrl.context.models[0].parameters()]).cpu(),
                       len(landed))
    assert out[False][1] == 0 and out[True][1] > 0
    torch.testing.assert_close(out[True][0], out[False][0], atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("rows,K,N", [(4608, 768, 2304), (4608, 3072, 768), (4608, 768, 768), (333, 128, 192),
                                      (200, 64, 128)])
def test_native_linear_exact_on_integer_operands(gpu, monkeypatch, rows, K, N):
    """DET_NATIVE_LINEAR: a Linear's forward (bias in the GEMM epilogue), input gradient (weight read
    as stored) and weight gradient on the det_conv.hip tiles, integer operands whose fp32 sums are
    exact: forward / input gradient bit-equal to the rounded fp32 product, weight gradient exact."""
    monkeypatch.setattr(tfops, "NATIVE_LINEAR", True)
    g = torch.Generator().manual_seed(rows + K + N)
    x = torch.randint(-2, 3, (rows, K), generator=g).to(torch.bfloat16)
    w = torch.randint(-2, 3, (N, K), generator=g).to(torch.bfloat16)
    b = torch.randint(-4, 5, (N,), generator=g).to(torch.bfloat16)
    dy = torch.randint(-2, 3, (rows, N), generator=g).to(torch.bfloat16)
    before = dict(tfops.LINEAR_COUNTS)
    xd, wd, bd = _leaf(x, gpu), _leaf(w, gpu), _leaf(b, gpu)
    y = tfops.linear(xd, wd, bd)
    y.backward(dy.to(gpu))
    assert all(tfops.LINEAR_COUNTS[k] == before[k] + 1 for k in before if k.startswith("native_")), tfops.LINEAR_COUNTS
    assert torch.equal(y.cpu(), (x.float() @ w.float().t() + b.float()).to(torch.bfloat16))
    assert torch.equal(xd.grad.cpu(), (dy.float() @ w.float()).to(torch.bfloat16))
    assert torch.equal(wd.grad.float().cpu(), (dy.float().t() @ x.float()).to(torch.bfloat16).float())
    torch.testing.assert_close(bd.grad.float().cpu(), dy.float().sum(0), rtol=1e-2, atol=1e-2)


def test_bert_layer_native_linear_matches_hipblaslt(gpu, monkeypatch):
    """The BERT encoder layer with its dense layers on the hand-written GEMMs vs on hipBLASLt."""
    from determined_1_amd.models.bert import BertEncoderConfig, BertLayer

    torch.manual_seed(0)
    cfg = BertEncoderConfig(hidden_size=256, num_attention_heads=4, intermediate_size=1024,
                            hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    layer = BertLayer(cfg)
    for name, p in layer.named_parameters():  # the BertForQA initialisation (torch.empty otherwise)
        with torch.no_grad():
            if name.endswith("weight") and p.dim() == 2:
                p.normal_(0.0, 0.02)
            elif "ln" in name and name.endswith("weight"):
                p.fill_(1.0)
            else:
                p.normal_(0.0, 0.02)
    layer = layer.to(gpu).to(torch.bfloat16)
    x = torch.randn(2, 128, 256, device=gpu).to(torch.bfloat16)
    mask = torch.zeros(2, 1, 1, 128, device=gpu, dtype=torch.bfloat16)
    outs = {}
    for native in (False, True):
        monkeypatch.setattr(tfops, "NATIVE_LINEAR", native)
        layer.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        y = layer(xi, mask)
        y.float().square().sum().backward()
        outs[native] = (y.float(), xi.grad.float(), {k: p.grad.float() for k, p in layer.named_parameters()})
    (y0, dx0, g0), (y1, dx1, g1) = outs[False], outs[True]
    torch.testing.assert_close(y1, y0, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(dx1, dx0, rtol=5e-2, atol=5e-2 * float(dx0.abs().max()))
    for k in g0:
        rel = float((g1[k] - g0[k]).norm() / (g0[k].norm() + 1e-12))
        assert rel < 3e-2, (k, rel)


def test_residual_gradient_link_sums_in_the_gemm(gpu, monkeypatch):
    """The BERT layer's input and its attention output are each read by a Linear and as a later
    LayerNorm residual: their two gradients meet in the Linear's input-gradient GEMM (the LayerNorm
    backward parks its residual gradient on a ResidualGradLink, the GEMM accumulates onto it) instead
    of autograd's separate add.  fp32: equal to the unlinked layer; both links really carry a gradient."""
    from determined_1_amd.models.bert import BertEncoderConfig, BertLayer

    torch.manual_seed(1)
    cfg = BertEncoderConfig(hidden_size=256, num_attention_heads=4, intermediate_size=1024,
                            hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    layer = BertLayer(cfg)
    with torch.no_grad():
        for p in layer.parameters():
            p.normal_(0.0, 0.05)
    layer = layer.to(gpu)
    x = torch.randn(2, 96, 256, device=gpu)
    mask = torch.zeros(2, 1, 1, 96, device=gpu)
    taken = []
    orig_take = tfops.ResidualGradLink.take

    def take(self):
        dr = orig_take(self)
        taken.append(dr is not None)
        return dr

    monkeypatch.setattr(tfops.ResidualGradLink, "take", take)
    outs = {}
    for linked in (True, False):
        if not linked:
            monkeypatch.setattr(tfops, "_arm", lambda link, x: None)
        layer.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        y = layer(xi, mask)
        y.square().sum().backward()
        outs[linked] = (xi.grad.clone(), {k: p.grad.clone() for k, p in layer.named_parameters()})
    assert taken[:2] == [True, True], taken
    torch.testing.assert_close(outs[True][0], outs[False][0], rtol=1e-5, atol=1e-5)
    for k in outs[False][1]:
        torch.testing.assert_close(outs[True][1][k], outs[False][1][k], rtol=1e-5, atol=1e-5, msg=k)


def test_tuned_gemm_solutions_load_and_keep_numerics(gpu, monkeypatch):
    """The measured hipBLASLt / rocBLAS solutions (ops/gemm_tuning.py, opt-in) load read-only on
    gfx950, and the tuned weight-gradient shape of BERT-base (reduction over 4608 tokens) stays
    within bf16 accuracy of the fp32 product."""
    from determined_1_amd.ops import gemm_tuning

    monkeypatch.setenv("DET_TUNED_GEMMS", "1")
    monkeypatch.setitem(gemm_tuning._STATE, "loaded", None)
    assert gemm_tuning.enable()
    assert torch.cuda.tunable.is_enabled() and not torch.cuda.tunable.tuning_is_enabled()
    g = torch.Generator(device=gpu).manual_seed(0)
    dz = torch.randn(4608, 3072, device=gpu, generator=g).to(torch.bfloat16)
    x = torch.randn(4608, 768, device=gpu, generator=g).to(torch.bfloat16)
    w = dz.t() @ x
    ref = dz.float().t() @ x.float()
    assert float((w.float() - ref).norm() / ref.norm()) < 1e-2
    # the measured solution (not the heuristic) served that shape
    res = {(r[0], r[1]): r[2] for r in torch.cuda.tunable.get_results()}
    assert res.get(("GemmTunableOp_BFloat16_NT", "nt_3072_768_4608_ld_3072_768_3072"), "").startswith("Gemm_"), res
    y = torch.addmm(torch.zeros(2304, device=gpu, dtype=torch.bfloat16), x, torch.randn(2304, 768, device=gpu,
                    generator=g).to(torch.bfloat16).t())
    assert bool(torch.isfinite(y).all())


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_blaslt_plans_match_torch_gemms(gpu, dt):
    """The cached-plan hipBLASLt path (ops/csrc/det_blaslt.hip) for the three Linear passes at a
    BERT shape -- forward with the bias epilogue, input gradient (alone and accumulated onto a
    residual gradient, beta = 1), weight gradient (alone and accumulated) -- against the fp32
    products, and against torch's own hipBLASLt calls to bf16 rounding."""
    M, K, N = 4608, 768, 2304
    g = torch.Generator(device=gpu).manual_seed(2)
    x = torch.randn(M, K, device=gpu, generator=g).to(dt)
    w = (torch.randn(N, K, device=gpu, generator=g) * 0.05).to(dt)
    b = torch.randn(N, device=gpu, generator=g).to(dt)
    dz = torch.randn(M, N, device=gpu, generator=g).to(dt)
    dr = torch.randn(M, K, device=gpu, generator=g).to(dt)
    assert tfops._bl_ok(x, w)
    tol = dict(rtol=2e-2, atol=2e-2) if dt == torch.bfloat16 else dict(rtol=1e-4, atol=1e-3)

    def close(a, ref):
        torch.testing.assert_close(a.float(), ref, **tol)

    y = torch.empty(M, N, device=gpu, dtype=dt)
    tfops._bl_gemm(1, 0, N, M, K, w, K, x, K, y, N, bias=b)
    close(y, x.float() @ w.float().t() + b.float())
    close(y, torch.addmm(b, x, w.t()).float())
    dx = torch.empty(M, K, device=gpu, dtype=dt)
    tfops._bl_gemm(0, 0, K, M, N, w, K, dz, N, dx, K)
    close(dx, dz.float() @ w.float())
    acc = dr.clone()
    tfops._bl_gemm(0, 0, K, M, N, w, K, dz, N, acc, K, beta=1.0)
    close(acc, dr.float() + dz.float() @ w.float())
    dw = torch.empty(N, K, device=gpu, dtype=dt)
    tfops._bl_wgrad(dz, x, dw)
    close(dw, dz.float().t() @ x.float())
    close(dw, (dz.t() @ x).float())
    tfops._bl_wgrad(dz, x, dw, beta=1.0)
    close(dw, 2 * (dz.float().t() @ x.float()))


@pytest.mark.parametrize("rows,K,N", [(4608, 768, 2304), (333, 128, 192)])
def test_linear_bias_grad_from_gemm_epilogue(gpu, monkeypatch, rows, K, N):
    """ops.transformer.linear's bias gradient from the weight-gradient GEMM's epilogue (hipBLASLt
    BGRADB) equals the column sums of dy (the separate det_tf_colsum pass it replaces); a shape the
    library cannot do that for falls back to the column sum, counted either way."""
    monkeypatch.setattr(tfops, "NATIVE_LINEAR", False)
    g = torch.Generator().manual_seed(rows + N)
    x = torch.randn(rows, K, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, generator=g).to(torch.bfloat16)
    dy = torch.randn(rows, N, generator=g).to(torch.bfloat16)
    res = {}
    for on in (False, True):
        monkeypatch.setattr(tfops, "BGRAD_EPILOGUE", on)
        before = dict(tfops.LINEAR_BGRAD_COUNTS)
        xd, wd, bd = _leaf(x, gpu), _leaf(w, gpu), _leaf(b, gpu)
        tfops.linear(xd, wd, bd).backward(dy.to(gpu))
        used = tfops.LINEAR_BGRAD_COUNTS["epilogue"] - before["epilogue"]
        assert used + tfops.LINEAR_BGRAD_COUNTS["colsum"] - before["colsum"] == 1
        if not on:
            assert used == 0
        res[on] = (bd.grad.float().cpu(), wd.grad.float().cpu(), xd.grad.float().cpu())
    ref = dy.float().sum(0)
    torch.testing.assert_close(res[True][0], ref, rtol=2e-2, atol=0.5)
    torch.testing.assert_close(res[False][0], ref, rtol=2e-2, atol=0.5)
    # the epilogue plan may use another algorithm (accumulation order) for the weight gradient
    torch.testing.assert_close(res[True][1], res[False][1], rtol=2e-2, atol=2e-2 * float(res[False][1].abs().max()))
    assert torch.equal(res[True][2], res[False][2])
