"""Numerics of the 3x3 conv path (ops.conv.conv_rs / _ConvRS on det_igemm v2/v3 + det_conv's
im2col weight gradient) against plain PyTorch fp32 references: every det_igemm tile configuration
on ragged / strided / padded shapes, exact small-integer operands (a tap, row or swizzle mix-up
shows exactly), BN statistics partials of the 256- and 512-row block variants, the weight
gradient, and the autograd function end to end with its FALLBACK counters."""
import pytest
import torch
import torch.nn.functional as F

from determined_1_amd.ops import _lib, conv

pytestmark = pytest.mark.gpu

CFG_SHAPES = [  # (Nb, Cin, H, W, Cout, R, stride, pad)
    (3, 128, 7, 9, 128, 3, 1, 1),      # M = 189 < one block
    (2, 256, 15, 15, 256, 3, 2, 1),    # stride 2, odd input
    (4, 64, 28, 28, 64, 3, 1, 1),      # N = 64, several blocks + tail
    (2, 512, 7, 7, 512, 3, 1, 1),
    (2, 256, 9, 9, 512, 1, 2, 0),      # 1x1 stride-2 gather
]


def _data(case, gpu, seed=0, integer=False):
    nb, cin, h, w, cout, r, st, pad = case
    g = torch.Generator(device="cpu").manual_seed(seed)
    if integer:
        x = torch.randint(-2, 3, (nb, cin, h, w), generator=g).to(torch.bfloat16)
        wt = torch.randint(-2, 3, (cout, cin, r, r), generator=g).to(torch.bfloat16)
    else:
        x = torch.randn(nb, cin, h, w, generator=g).to(torch.bfloat16)
        wt = (torch.randn(cout, cin, r, r, generator=g) / (cin * r * r) ** 0.5).to(torch.bfloat16)
    return x, wt, x.to(gpu).contiguous(memory_format=torch.channels_last), wt.to(gpu).contiguous(
        memory_format=torch.channels_last)


def _run_cfg(xg, wg, st, pad, cfg, stats=False):
    try:
        return conv.igemm_conv(xg, wg, stride=st, pad=pad, cfg=cfg, stats=stats)
    except RuntimeError as e:
        if "-6" in str(e) or "-7" in str(e):
            pytest.skip(f"cfg {cfg} does not cover this shape")
        raise


@pytest.mark.parametrize("cfg", list(range(1, 16)) + [21, 22])
@pytest.mark.parametrize("case", CFG_SHAPES)
def test_every_cfg_exact_on_integer_operands(gpu, case, cfg):
    nb, cin, h, w, cout, r, st, pad = case
    x, wt, xg, wg = _data(case, gpu, integer=True)
    y, _ = _run_cfg(xg, wg, st, pad, cfg)
    ref = F.conv2d(x.float(), wt.float(), stride=st, padding=pad)
    assert y.is_contiguous(memory_format=torch.channels_last)
    # integer sums up to 9 * 512 * 4 = 18432 are exact in fp32; bf16 rounds above 256
    torch.testing.assert_close(y.float().cpu(), ref.to(torch.bfloat16).float(), rtol=0, atol=0)


@pytest.mark.parametrize("cfg", [0, 2, 8, 11, 13, 21, 22])
def test_cfg_stats_partials(gpu, cfg):
    case = (4, 256, 28, 28, 256, 3, 1, 1)  # M = 3136: ragged last block for 256 and 512 rows
    nb, cin, h, w, cout, r, st, pad = case
    _, _, xg, wg = _data(case, gpu, seed=3)
    y, (pm, pq, rpb) = _run_cfg(xg, wg, st, pad, cfg, stats=True)
    yr = y.permute(0, 2, 3, 1).reshape(-1, cout).double().cpu()
    m = yr.shape[0]
    nrb = pm.shape[0]
    assert nrb == (m + rpb - 1) // rpb and rpb == int(_lib.get_lib().det_igemm_rows_per_block_cfg(cout, cfg))
    cnt = torch.full((nrb, 1), float(rpb), dtype=torch.float64)
    cnt[-1, 0] = float(m - (nrb - 1) * rpb)
    pmd, pqd = pm.double().cpu(), pq.double().cpu()
    mean = (pmd * cnt).sum(0) / m
    var = (pqd + cnt * (pmd - mean) ** 2).sum(0) / m
    torch.testing.assert_close(mean, yr.mean(0), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(var, yr.var(0, unbiased=False), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("case", [(3, 64, 9, 11, 128, 3, 1, 1), (2, 128, 15, 15, 128, 3, 2, 1),
                                  (2, 256, 7, 7, 64, 3, 1, 1), (2, 128, 14, 14, 256, 1, 2, 0)])
def test_conv_wgrad_matches_torch(gpu, case):
    nb, cin, h, w, cout, r, st, pad = case
    x, wt, xg, _ = _data(case, gpu, seed=7)
    ho = (h + 2 * pad - r) // st + 1
    g = torch.Generator(device="cpu").manual_seed(8)
    dy = torch.randn(nb, cout, ho, (w + 2 * pad - r) // st + 1, generator=g).to(torch.bfloat16)
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, r, r), dy.float(), stride=st, padding=pad)
    for dt in (torch.float32, torch.bfloat16):
        out = torch.empty(cout, r * r * cin, dtype=dt, device=gpu)
        conv.conv_wgrad(dy.to(gpu).contiguous(memory_format=torch.channels_last), xg, out, r, r, st, pad)
        got = out.view(cout, r, r, cin).permute(0, 3, 1, 2).float().cpu()
        tol = 1e-3 if dt == torch.float32 else 1e-2
        torch.testing.assert_close(got, ref, rtol=tol, atol=tol * float(ref.abs().max()))


WGRAD_SHAPES = [  # (Nb, Cin, H, W, Cout, R, stride, pad)
    (3, 64, 9, 11, 64, 3, 1, 1),       # M = 297: ragged last K step
    (8, 64, 28, 28, 64, 3, 1, 1),      # many splits, multi-row pixel carries
    (2, 128, 15, 15, 128, 3, 2, 1),    # stride 2, odd input
    (2, 256, 7, 7, 256, 3, 1, 1),      # Ho*Wo = 49 > 32: image carries inside a step
    (2, 128, 14, 14, 256, 1, 2, 0),    # 1x1 stride-2
    (4, 256, 7, 7, 64, 1, 1, 0),       # 1x1, N = 64
    (3, 256, 10, 9, 256, 3, 2, 1),     # 256 x 256 tiles (wgrad8): stride 2, ragged K tail
    (1, 512, 5, 7, 512, 3, 1, 1),      # 256 x 256 tiles, M = 35 < one K tile
    (2, 256, 9, 9, 512, 1, 1, 0),      # 1x1, N = 512, RSC = 256
]


@pytest.mark.parametrize("cfg", list(range(1, 15)))
@pytest.mark.parametrize("case", WGRAD_SHAPES)
def test_ring_wgrad_every_cfg_exact(gpu, case, cfg):
    """det_igemm_wgrad (LDS-DMA ring + transposed reads) per tile configuration on small-integer
    operands: every product and partial sum is exact in fp32, so any tap / swizzle / split /
    carry error shows as an exact mismatch against torch's fp32 weight gradient."""
    nb, cin, h, w, cout, r, st, pad = case
    x, _, xg, _ = _data(case, gpu, seed=5, integer=True)
    ho, wo = (h + 2 * pad - r) // st + 1, (w + 2 * pad - r) // st + 1
    g = torch.Generator(device="cpu").manual_seed(6)
    dy = torch.randint(-2, 3, (nb, cout, ho, wo), generator=g).to(torch.bfloat16)
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, r, r), dy.float(), stride=st, padding=pad)
    out = torch.full((cout, r * r * cin), float("nan"), dtype=torch.float32, device=gpu)
    before = dict(conv.WGRAD_COUNTS)
    try:
        conv.conv_wgrad(dy.to(gpu).contiguous(memory_format=torch.channels_last), xg, out, r, r, st, pad, cfg=cfg)
    except RuntimeError as e:
        if "-6" in str(e):
            pytest.skip(f"wgrad cfg {cfg} does not cover this shape")
        raise
    assert conv.WGRAD_COUNTS["ring"] == before["ring"] + 1
    got = out.view(cout, r, r, cin).permute(0, 3, 1, 2).cpu()
    torch.testing.assert_close(got, ref, rtol=0, atol=0)


def test_ring_wgrad_scale_and_bf16_out(gpu):
    case = (4, 128, 14, 14, 128, 3, 1, 1)
    nb, cin, h, w, cout, r, st, pad = case
    x, _, xg, _ = _data(case, gpu, seed=9)
    g = torch.Generator(device="cpu").manual_seed(10)
    dy = torch.randn(nb, cout, h, w, generator=g).to(torch.bfloat16)
    ref = 0.25 * torch.nn.grad.conv2d_weight(x.float(), (cout, cin, r, r), dy.float(), stride=st, padding=pad)
    out = torch.empty(cout, r * r * cin, dtype=torch.bfloat16, device=gpu)
    conv.conv_wgrad(dy.to(gpu).contiguous(memory_format=torch.channels_last), xg, out, r, r, st, pad, out_scale=0.25)
    got = out.view(cout, r, r, cin).permute(0, 3, 1, 2).float().cpu()
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))


def test_dgrad_weight_kernel_matches_torch(gpu):
    for dt in (torch.float32, torch.bfloat16):
        w = torch.randn(96, 64, 3, 3, device=gpu).to(dt).contiguous(memory_format=torch.channels_last)
        got = conv.dgrad_weight(w)
        ref = w.flip(2, 3).permute(1, 2, 3, 0).reshape(64, -1).to(torch.bfloat16)
        assert torch.equal(got, ref)


def test_dgrad_weight_multi_matches_single_flips(gpu, monkeypatch):
    """det_conv_dgrad_weight_multi: every weight registered by a forward flipped in ONE launch at the
    backward's first dgrad_weight call, bit-equal to the torch flip (40 weights: two 32-entry chunks)."""
    monkeypatch.setattr(conv, "DW_BATCH", True)
    conv._DW_PENDING.clear()
    conv._DW_READY.clear()
    torch.manual_seed(0)
    shapes = [(64, 64, 3, 3), (128, 128, 3, 3), (512, 512, 3, 3), (96, 192, 3, 3), (64, 8, 7, 7), (200, 72, 5, 5)]
    ws = []
    for i in range(40):
        k, c, r, s = shapes[i % len(shapes)]
        dt = torch.bfloat16 if i % 3 else torch.float32
        ws.append(torch.randn(k, c, r, s, device=gpu).to(dt).contiguous(memory_format=torch.channels_last))
    for w in ws:
        conv.dgrad_weight_register(w)
    b0, s0 = conv.DW_COUNTS["batched_launches"], conv.DW_COUNTS["served"]
    for w in reversed(ws):  # backward order
        k, c, r, s = w.shape
        ref = w.flip(2, 3).permute(1, 2, 3, 0).reshape(c, -1).to(torch.bfloat16)
        assert torch.equal(conv.dgrad_weight(w), ref)
    assert conv.DW_COUNTS["batched_launches"] == b0 + 1
    assert conv.DW_COUNTS["served"] == s0 + len(ws)
    assert not conv._DW_PENDING and not conv._DW_READY


def test_batched_flips_follow_in_place_weight_updates(gpu, monkeypatch):
    """Three forward/backward steps of two 3x3 convs with the weights changed in place between steps
    (as the fused optimizer does, without a version bump): every input gradient uses the weights of
    its own forward."""
    monkeypatch.setattr(conv, "DW_BATCH", True)
    torch.manual_seed(1)
    m1 = torch.nn.Conv2d(64, 64, 3, padding=1, bias=False).to(gpu).to(torch.bfloat16).to(memory_format=torch.channels_last)
    m2 = torch.nn.Conv2d(64, 64, 3, padding=1, bias=False).to(gpu).to(torch.bfloat16).to(memory_format=torch.channels_last)
    for step in range(3):
        x = torch.randn(2, 64, 14, 14, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x.requires_grad_(True)
        b0 = conv.DW_COUNTS["batched_launches"]
        y = conv.conv_rs(conv.conv_rs(x, m1), m2)
        dy = torch.randn_like(y)
        y.backward(dy)
        assert conv.DW_COUNTS["batched_launches"] == b0 + 1  # both flips in one launch
        xr = x.detach().float().requires_grad_(True)
        yr = F.conv2d(F.conv2d(xr, m1.weight.detach().float(), padding=1).to(torch.bfloat16).float(),
                      m2.weight.detach().float(), padding=1)
        yr.backward(dy.float())
        torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=2e-2 * float(xr.grad.abs().max()))
        with torch.no_grad():  # in-place update through the raw storage: no version counter change
            m1.weight.data.copy_(torch.randn_like(m1.weight) * 0.05)
            m2.weight.data.copy_(torch.randn_like(m2.weight) * 0.05)


@pytest.mark.parametrize("wgrad_mode", ["miopen", "auto", "native"])
@pytest.mark.parametrize("stride", [1, 2])
def test_conv_rs_autograd_end_to_end(gpu, stride, wgrad_mode, monkeypatch):
    monkeypatch.setattr(conv, "WGRAD_RS_MODE", wgrad_mode)
    native_wgrad = wgrad_mode in ("native", "auto")  # auto: conv3p_wgrad at stride 1, the ring at stride 2
    torch.manual_seed(0)
    m = torch.nn.Conv2d(128, 128, 3, stride=stride, padding=1, bias=False).to(gpu).to(
        memory_format=torch.channels_last)
    x = torch.randn(4, 128, 14, 14, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    before = dict(conv.CONV3X3_COUNTS)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = conv.conv_rs(x, m)
    dy = torch.randn_like(y)
    y.backward(dy)
    assert conv.CONV3X3_COUNTS["native"] == before["native"] + 1
    assert conv.CONV3X3_COUNTS["fallback"] == before["fallback"]
    wkey = "wgrad_native" if native_wgrad else "wgrad_miopen"
    assert conv.CONV3X3_COUNTS[wkey] == before[wkey] + 1
    assert conv.CONV3X3_COUNTS["dgrad_native"] == before["dgrad_native"] + 1  # stride 2: parity classes
    assert conv.CONV3X3_COUNTS["dgrad_miopen"] == before["dgrad_miopen"]
    xr = x.detach().float().requires_grad_(True)
    wr = m.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=stride, padding=1)
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(m.weight.grad.float(), wr.grad, rtol=2e-2, atol=2e-2 * float(wr.grad.abs().max()))


S2_SHAPES = [  # (Nb, Cout, Ho, Wo, Cin): ResNet's three stride-2 3x3 convs (reduced batch) + ragged tails
    (2, 128, 28, 28, 128),
    (3, 256, 14, 14, 256),
    (2, 512, 7, 7, 512),
    (1, 64, 5, 9, 192),    # Cin 192 -> BN 64 tiles, odd output grid, M < one block
]


@pytest.mark.parametrize("case", S2_SHAPES)
def test_dgrad_s2_exact_on_integer_operands(gpu, case):
    """det_igemm_dgrad_s2 (four parity-class implicit GEMMs over dY) == conv2d_input of the stride-2
    3x3 conv, exactly: small-integer operands keep every sum exact in fp32, so a wrong tap, class
    scatter or row offset shows as a mismatch."""
    nb, cout, ho, wo, cin = case
    g = torch.Generator(device="cpu").manual_seed(11)
    dy = torch.randint(-2, 3, (nb, cout, ho, wo), generator=g).to(torch.bfloat16)
    wt = torch.randint(-2, 3, (cout, cin, 3, 3), generator=g).to(torch.bfloat16)
    ref = torch.nn.grad.conv2d_input((nb, cin, 2 * ho, 2 * wo), wt.float(), dy.float(), stride=2, padding=1)
    got = conv.igemm_dgrad_s2(dy.to(gpu).contiguous(memory_format=torch.channels_last),
                              wt.to(gpu).contiguous(memory_format=torch.channels_last), 2 * ho, 2 * wo)
    assert got.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(got.float().cpu(), ref.to(torch.bfloat16).float(), rtol=0, atol=0)


def test_dgrad_s2_bn_backward_epilogue_matches_unfused(gpu):
    """The fused path: the BN(+ReLU) that produced the stride-2 conv's input takes its backward
    partials from the class GEMMs' epilogue; x.grad, dgamma, dbeta equal the unfused backward."""
    from determined_1_amd.ops import norm

    torch.manual_seed(2)
    bn = norm.BatchNormAct2d(128, relu=True).to(gpu)
    m = torch.nn.Conv2d(128, 128, 3, stride=2, padding=1, bias=False).to(gpu).to(memory_format=torch.channels_last)
    x0 = torch.randn(4, 128, 28, 28, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = None
    outs = []
    for fuse in (False, True):
        conv.FUSE_BN_BWD = fuse
        try:
            bn.zero_grad(set_to_none=True)
            m.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            before = dict(conv.BN_BWD_COUNTS)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = conv.conv_rs(bn(x), m, bn_exclusive=True)
            if dy is None:
                dy = torch.randn_like(y)
            y.backward(dy)
            if fuse:
                assert conv.BN_BWD_COUNTS["fused"] == before["fused"] + 1
            outs.append([x.grad.float(), bn.weight.grad, bn.bias.grad, m.weight.grad.float()])
        finally:
            conv.FUSE_BN_BWD = True
    for a, b in zip(*outs):
        torch.testing.assert_close(b, a, rtol=2e-2, atol=2e-2 * float(a.abs().max()) + 1e-6)


P3_SHAPES = [  # (Nb, Cin, H, W, Cout)
    (2, 64, 56, 56, 64),    # ResNet layer1 (reduced batch)
    (3, 128, 28, 28, 128),  # layer2: two N tiles per pixel tile
    (4, 64, 14, 14, 64),    # 256-pixel tiles span images (patch with per-image padding rows)
    (1, 32, 7, 9, 64),      # Cin 32 (one slice), odd width, M < one tile
    (6, 64, 7, 7, 128),     # tiles spanning 5+ images
]


@pytest.mark.parametrize("case", P3_SHAPES)
def test_conv3p_exact_on_integer_operands(gpu, case):
    """det_conv3p (input staged once per tile as a halo patch, 9 taps read at row offsets) ==
    F.conv2d exactly on small-integer operands, with and without the BN+ReLU prologue (integer
    scale/shift keep it exact; the zero padding must not be transformed)."""
    nb, cin, h, w, cout = case
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randint(-2, 3, (nb, cin, h, w), generator=g).to(torch.bfloat16)
    wt = torch.randint(-2, 3, (cout, cin, 3, 3), generator=g).to(torch.bfloat16)
    xg = x.to(gpu).contiguous(memory_format=torch.channels_last)
    wk = conv.krsc(wt.to(gpu).contiguous(memory_format=torch.channels_last))
    y, _ = conv.conv3p(xg, wk, cout)
    ref = F.conv2d(x.float(), wt.float(), padding=1)
    torch.testing.assert_close(y.float().cpu(), ref.to(torch.bfloat16).float(), rtol=0, atol=0)
    sc = torch.randint(-1, 3, (cin,), generator=g).float()
    sh = torch.randint(-2, 2, (cin,), generator=g).float()
    yp, _ = conv.conv3p(xg, wk, cout, pro=(sc.to(gpu), sh.to(gpu)))
    z = torch.relu(x.float() * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1))
    refp = F.conv2d(z, wt.float(), padding=1)
    torch.testing.assert_close(yp.float().cpu(), refp.to(torch.bfloat16).float(), rtol=0, atol=0)


def test_conv3p_stats_and_bn_backward_epilogues(gpu):
    nb, cin, h, w, cout = 4, 64, 28, 28, 128  # M = 3136: ragged last 256-row block
    g = torch.Generator(device="cpu").manual_seed(9)
    x = (torch.randn(nb, cin, h, w, generator=g)).to(torch.bfloat16)
    wt = (torch.randn(cout, cin, 3, 3, generator=g) / 24).to(torch.bfloat16)
    xg = x.to(gpu).contiguous(memory_format=torch.channels_last)
    wk = conv.krsc(wt.to(gpu).contiguous(memory_format=torch.channels_last))
    y, (pm, pq, rpb) = conv.conv3p(xg, wk, cout, stats=True)
    yr = y.permute(0, 2, 3, 1).reshape(-1, cout).double().cpu()
    m = yr.shape[0]
    cnt = torch.full((pm.shape[0], 1), float(rpb), dtype=torch.float64)
    cnt[-1, 0] = float(m - (pm.shape[0] - 1) * rpb)
    mean = (pm.double().cpu() * cnt).sum(0) / m
    var = (pq.double().cpu() + cnt * (pm.double().cpu() - mean) ** 2).sum(0) / m
    torch.testing.assert_close(mean, yr.mean(0), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(var, yr.var(0, unbiased=False), rtol=1e-4, atol=1e-5)
    # BNB: the output is the gradient reaching a BN(+ReLU) with input bx: masked, with partial sums
    bx = torch.randn(nb, cout, h, w, generator=g).to(torch.bfloat16).to(gpu).contiguous(memory_format=torch.channels_last)
    bmean = torch.randn(cout, generator=g).to(gpu)
    bsc = torch.rand(cout, generator=g).add(0.5).to(gpu)
    bsh = torch.randn(cout, generator=g).to(gpu)
    d, (ps, psx, _) = conv.conv3p(xg, wk, cout, bnb=(bx, bmean, bsc, bsh))
    mask = (bx.float() * bsc.view(1, -1, 1, 1) + bsh.view(1, -1, 1, 1)) > 0
    want = torch.where(mask, y.float(), torch.zeros_like(y.float())).to(torch.bfloat16)
    assert torch.equal(d, want)
    df = d.float().permute(0, 2, 3, 1).reshape(-1, cout).double()
    xf = bx.float().permute(0, 2, 3, 1).reshape(-1, cout).double()
    torch.testing.assert_close(ps.double().sum(0), df.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(psx.double().sum(0), (df * (xf - bmean.double())).sum(0), rtol=1e-4, atol=1e-3)


def test_conv_rs_routes_thin_3x3_to_conv3p(gpu, monkeypatch):
    """The autograd 3x3 path runs conv3p for N <= CONV3P_MAX_N (forward and stride-1 dgrad) and the
    result matches the fp32 reference (conv3p is opt-in: DET_CONV3P_MAX_N)."""
    monkeypatch.setattr(conv, "CONV3P_MAX_N", 128)
    torch.manual_seed(0)
    m = torch.nn.Conv2d(64, 64, 3, padding=1, bias=False).to(gpu).to(memory_format=torch.channels_last)
    x = torch.randn(4, 64, 28, 28, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    before = dict(conv.CONV3P_COUNTS)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = conv.conv_rs(x, m)
    dy = torch.randn_like(y)
    y.backward(dy)
    # the forward and the (unfused: no BN producer) stride-1 input gradient both run conv3p
    assert conv.CONV3P_COUNTS["fwd"] == before["fwd"] + 2
    xr = x.detach().float().requires_grad_(True)
    wr = m.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    yr = F.conv2d(xr, wr, padding=1)
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=3e-2)


WP_SHAPES = [  # (Nb, Cin, H, W, Cout)
    (2, 64, 56, 56, 64),
    (3, 128, 28, 28, 128),  # 2 x 2 weight tiles
    (4, 64, 14, 14, 128),   # chunks spanning images
    (1, 64, 7, 9, 64),      # one partial chunk
]


@pytest.mark.parametrize("case", WP_SHAPES)
def test_conv3p_wgrad_exact_on_integer_operands(gpu, case):
    """det_conv3p_wgrad (dY and the input patch staged once per 256 pixels for all 9 taps, transposed
    reads at per-lane patch rows) == torch's conv2d_weight exactly on small-integer operands (sums
    stay exact in fp32; fp32 output)."""
    nb, cin, h, w, cout = case
    g = torch.Generator(device="cpu").manual_seed(13)
    x = torch.randint(-2, 3, (nb, cin, h, w), generator=g).to(torch.bfloat16)
    dy = torch.randint(-2, 3, (nb, cout, h, w), generator=g).to(torch.bfloat16)
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, 3, 3), dy.float(), padding=1)
    out = torch.empty(cout, 9 * cin, dtype=torch.float32, device=gpu)
    assert conv.conv3p_wgrad(dy.to(gpu).contiguous(memory_format=torch.channels_last),
                             x.to(gpu).contiguous(memory_format=torch.channels_last), out)
    got = out.view(cout, 3, 3, cin).permute(0, 3, 1, 2).cpu()
    torch.testing.assert_close(got, ref, rtol=0, atol=0)
