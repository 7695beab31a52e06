"""Numerics of the hand-written 1x1-conv MFMA GEMMs (ops/csrc/det_conv.hip) against plain PyTorch
fp32 references of the same ops: forward (+ fused BN statistics, + BN-apply/ReLU prologue,
+ stride-2 row gather), dgrad through the transposed weight, and split-M wgrad."""
import pytest
import torch

from determined_1_amd.ops import conv

pytestmark = pytest.mark.gpu

SHAPES = [  # (M, Cin, Cout): ResNet-50 1x1 channel pairs at small M, incl. ragged row tails
    (1000, 64, 64), (777, 256, 64), (4096 + 77, 64, 256), (2048, 512, 128), (1500, 128, 512),
    (640, 1024, 256), (333, 512, 2048),
]


def _merge(pm, pq, rpb, m):
    nrb = pm.shape[0]
    cnt = torch.full((nrb, 1), float(rpb), dtype=torch.float64)
    cnt[-1, 0] = float(m - (nrb - 1) * rpb)
    pm, pq = pm.double().cpu(), pq.double().cpu()
    mean = (pm * cnt).sum(0) / m
    m2 = (pq + cnt * (pm - mean) ** 2).sum(0)
    return mean, m2 / m


@pytest.mark.parametrize("m,cin,cout", SHAPES)
@pytest.mark.parametrize("pro", [False, True])
def test_conv_nt_forward_stats(gpu, m, cin, cout, pro):
    torch.manual_seed(m + cin)
    x = torch.randn(m, cin, device=gpu).to(torch.bfloat16)
    w = (torch.randn(cout, cin, device=gpu) / cin ** 0.5).to(torch.bfloat16)
    scale = shift = None
    xa = x.float()
    if pro:
        scale = torch.rand(cin, device=gpu) + 0.5
        shift = torch.randn(cin, device=gpu) * 0.3
        xa = torch.relu(x.float() * scale + shift).to(torch.bfloat16).float()
    y, parts = conv.conv1x1_nt(x, w, scale=scale, shift=shift, stats=True)
    ref = xa @ w.float().t()
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    mean, var = _merge(*parts, m)
    yr = y.double().cpu()
    torch.testing.assert_close(mean, yr.mean(0), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(var, yr.var(0, unbiased=False), rtol=1e-4, atol=1e-5)


def test_conv_nt_asymmetric_exact(gpu):
    """Integer operands (exact in bf16 and fp32): any row/column mix-up of the MFMA maps shows."""
    m, k, n = 256 + 13, 128, 192
    a = torch.randint(-3, 4, (m, k), device=gpu).to(torch.bfloat16)
    b = torch.randint(-3, 4, (n, k), device=gpu).to(torch.bfloat16)
    b[:, 0] = torch.arange(n, device=gpu).to(torch.bfloat16) % 7
    y, _ = conv.conv1x1_nt(a, b)
    assert torch.equal(y.float(), a.float() @ b.float().t())


def test_conv_nt_stride2_gather(gpu):
    n_, hi, wi, cin, cout = 3, 14, 14, 256, 512
    x = torch.randn(n_, hi, wi, cin, device=gpu).to(torch.bfloat16)
    w = (torch.randn(cout, cin, device=gpu) / cin ** 0.5).to(torch.bfloat16)
    ho, wo = hi // 2, wi // 2
    m = n_ * ho * wo
    y, parts = conv.conv1x1_nt(x.view(-1, cin), w, m=m, stats=True, gather=(ho, wo, hi, wi))
    ref = x[:, ::2, ::2, :].reshape(m, cin).float() @ w.float().t()
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("m,cin,cout", SHAPES)
def test_conv_dgrad_via_transposed_weight(gpu, m, cin, cout):
    dy = torch.randn(m, cout, device=gpu).to(torch.bfloat16)
    w = (torch.randn(cout, cin, device=gpu) / cout ** 0.5).to(torch.bfloat16)
    dx, _ = conv.conv1x1_nt(dy, w.t().contiguous())
    torch.testing.assert_close(dx.float(), dy.float() @ w.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("m,cin,cout", SHAPES + [(777, 128, 64), (4096, 64, 64)])
def test_conv_dgrad_untransposed_weight_exact(gpu, m, cin, cout):
    """det_conv_dgrad (weight read as stored with transposed LDS reads) on small-integer operands:
    exact against the fp32 product, so a swizzle or k/n mix-up shows as a mismatch."""
    g = torch.Generator(device="cpu").manual_seed(m + cin)
    dy = torch.randint(-2, 3, (m, cout), generator=g).to(torch.bfloat16)
    w = torch.randint(-2, 3, (cout, cin), generator=g).to(torch.bfloat16)
    dx = conv.dgrad_1x1(dy.to(gpu), w.to(gpu))
    torch.testing.assert_close(dx.float().cpu(), (dy.float() @ w.float()).to(torch.bfloat16).float(), rtol=0, atol=0)


@pytest.fixture
def nt_pf():
    from determined_1_amd.ops import _lib

    lib = _lib.get_lib()
    yield lib.det_conv_nt_set_pf
    lib.det_conv_nt_set_pf(0)


PF_SHAPES = [  # (M, K, N): K tiles 2..10 cover every prefetch-ring phase at depths 1-3
    (777, 128, 256), (1000, 192, 128), (4096 + 77, 256, 512), (640, 320, 64), (1500, 512, 128), (333, 640, 256),
]


@pytest.mark.parametrize("pf", [1, 2, 3])
@pytest.mark.parametrize("m,k,n", PF_SHAPES)
def test_conv_nt_prefetch_depths_exact(gpu, nt_pf, pf, m, k, n):
    """det_conv_nt / det_conv_dgrad at every register prefetch depth (the K-tile ring of the plain
    GEMMs): integer operands whose fp32 sums are exact, so the bf16 output must equal the rounded
    fp32 product bit for bit -- a ring slot staged from the wrong K tile shows."""
    nt_pf(pf)
    g = torch.Generator(device="cpu").manual_seed(m + k + pf)
    a = torch.randint(-2, 3, (m, k), generator=g).to(torch.bfloat16)
    b = torch.randint(-2, 3, (n, k), generator=g).to(torch.bfloat16)
    want = (a.float() @ b.float().t()).to(torch.bfloat16)
    y, parts = conv.conv1x1_nt(a.to(gpu), b.to(gpu), stats=True)
    assert torch.equal(y.cpu(), want)
    mean, _ = _merge(*parts, m)
    torch.testing.assert_close(mean, y.double().cpu().mean(0), rtol=1e-6, atol=1e-6)
    # input gradient against the untransposed [K, N] weight (transposed LDS reads; depth capped at 2)
    dx = conv.dgrad_1x1(a.to(gpu), b.t().contiguous().to(gpu))
    assert torch.equal(dx.cpu(), want)


@pytest.mark.parametrize("m,k,n", [(777, 128, 512), (4096 + 77, 256, 1024), (1500, 512, 2048), (640, 128, 1024)])
def test_conv_nt_wide_tiles_exact(gpu, m, k, n):
    """The occupancy-3 128 x 64 tiles of the short-K wide-N forwards (det_conv_nt_set_wide): integer
    operands, exact against the fp32 product; statistics partials per 128 rows merge to the output's."""
    from determined_1_amd.ops import _lib

    lib = _lib.get_lib()
    g = torch.Generator(device="cpu").manual_seed(m + k)
    a = torch.randint(-2, 3, (m, k), generator=g).to(torch.bfloat16)
    b = torch.randint(-2, 3, (n, k), generator=g).to(torch.bfloat16)
    want = (a.float() @ b.float().t()).to(torch.bfloat16)
    lib.det_conv_nt_set_wide(1)
    try:
        y, parts = conv.conv1x1_nt(a.to(gpu), b.to(gpu), stats=True)
        y2, _ = conv.conv1x1_nt(a.to(gpu), b.to(gpu), stats=False)
    finally:
        lib.det_conv_nt_set_wide(-1)
    assert torch.equal(y.cpu(), want) and torch.equal(y2.cpu(), want)
    mean, var = _merge(*parts, m)
    yr = y.double().cpu()
    torch.testing.assert_close(mean, yr.mean(0), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(var, yr.var(0, unbiased=False), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("m,cin,cout", SHAPES + [(50000, 64, 256)])
@pytest.mark.parametrize("pro", [False, True])
def test_conv_wgrad(gpu, m, cin, cout, pro):
    torch.manual_seed(cin * 7 + cout)
    dy = torch.randn(m, cout, device=gpu).to(torch.bfloat16)
    x = torch.randn(m, cin, device=gpu).to(torch.bfloat16)
    scale = shift = None
    xa = x.float()
    if pro:
        scale = torch.rand(cin, device=gpu) + 0.5
        shift = torch.randn(cin, device=gpu) * 0.3
        xa = torch.relu(x.float() * scale + shift).to(torch.bfloat16).float()
    out = torch.empty(cout, cin, device=gpu, dtype=torch.float32)
    conv.conv1x1_wgrad(dy, x, out, scale=scale, shift=shift, out_scale=0.5)
    ref = (dy.float().t() @ xa) * 0.5
    torch.testing.assert_close(out, ref, rtol=1e-3, atol=1e-3 * m ** 0.5)
    outb = torch.empty(cout, cin, device=gpu, dtype=torch.bfloat16)
    conv.conv1x1_wgrad(dy, x, outb, scale=scale, shift=shift, out_scale=0.5)
    torch.testing.assert_close(outb.float(), out.to(torch.bfloat16).float(), rtol=1e-2, atol=1e-2)


def test_conv_wgrad_stride2(gpu):
    n_, hi, wi, cin, cout = 4, 14, 14, 512, 1024
    x = torch.randn(n_, hi, wi, cin, device=gpu).to(torch.bfloat16)
    ho, wo = hi // 2, wi // 2
    m = n_ * ho * wo
    dy = torch.randn(m, cout, device=gpu).to(torch.bfloat16)
    out = torch.empty(cout, cin, device=gpu, dtype=torch.float32)
    conv.conv1x1_wgrad(dy, x.view(-1, cin), out, gather=(ho, wo, hi, wi))
    ref = dy.float().t() @ x[:, ::2, ::2, :].reshape(m, cin).float()
    torch.testing.assert_close(out, ref, rtol=1e-3, atol=1e-3 * m ** 0.5)


def test_resnet50_native_conv1x1_matches_miopen(gpu):
    """Three SGD steps of ResNet-50 (bf16 O2-style: bf16 weights, fused BN) with the stride-1 1x1
    convs on det_conv GEMMs vs on MIOpen: same losses to bf16 tolerance, and the native path ran."""
    from determined_1_amd.models import resnet
    from determined_1_amd.ops import conv as nc

    def run(native):
        resnet.NATIVE_CONV1X1 = native
        torch.manual_seed(0)
        m = resnet.resnet50(num_classes=10).to(gpu).to(memory_format=torch.channels_last).to(torch.bfloat16)
        for mod in m.modules():  # BN params/buffers stay fp32 (keep_batchnorm_fp32)
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.float()
        opt = torch.optim.SGD(m.parameters(), lr=0.02, momentum=0.9)
        g = torch.Generator(device="cpu").manual_seed(1)
        x = torch.randn(8, 3, 64, 64, generator=g).to(gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (8,), generator=g).to(gpu)
        losses = []
        for _ in range(3):
            opt.zero_grad()
            loss = torch.nn.functional.cross_entropy(m(x).float(), y)
            loss.backward()
            opt.step()
            losses.append(float(loss))
        return losses

    before = nc.COUNTS["native"] + nc.FUSED_COUNTS["bn_relu_conv1x1"]
    ref = run(False)
    got = run(True)
    resnet.NATIVE_CONV1X1 = True
    # 32 stride-1 1x1 convs per ResNet-50 forward (conv3 of each block with bn2 in its prologue)
    assert nc.COUNTS["native"] + nc.FUSED_COUNTS["bn_relu_conv1x1"] - before >= 3 * 32
    for a, b in zip(got, ref):
        assert abs(a - b) < 0.05 * max(1.0, abs(b)), (got, ref)


@pytest.mark.parametrize("m,cout", [(65536 + 40, 256), (200704, 64)])
def test_conv_stats_feed_bn_two_stage_finalize(gpu, m, cout):
    """GEMM-epilogue statistics of a long activation (hundreds of 128-row partial blocks) through
    the two-stage BN finalize: batch mean/var, running stats and the normalized output match
    torch.batch_norm on the same bf16 conv output."""
    from determined_1_amd.ops import norm

    torch.manual_seed(3)
    cin = 64
    x = (torch.randn(m, cin, device=gpu) + 0.3).to(torch.bfloat16)
    w = (torch.randn(cout, cin, device=gpu) / cin ** 0.5).to(torch.bfloat16)
    conv_mod = torch.nn.Conv2d(cin, cout, 1, bias=False).to(gpu).to(torch.bfloat16)
    with torch.no_grad():
        conv_mod.weight.copy_(w.view(cout, cin, 1, 1))
    x4 = x.view(1, m, 1, cin).permute(0, 3, 1, 2)  # channels_last view [1, cin, m, 1]
    bn = norm.BatchNormAct2d(cout, relu=False, fused=True).to(gpu)
    ref_bn = norm.BatchNormAct2d(cout, relu=False, fused=False).to(gpu)
    with torch.no_grad():
        y = conv.conv1x1(x4, conv_mod)
        out = bn(y)
        yr = (x.float() @ w.float().t()).to(torch.bfloat16).float().view(1, m, 1, cout).permute(0, 3, 1, 2)
        ref = torch.nn.functional.batch_norm(yr, ref_bn.running_mean, ref_bn.running_var, None, None, True, 0.1, bn.eps)
    torch.testing.assert_close(bn.running_mean, ref_bn.running_mean, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(bn.running_var, ref_bn.running_var, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=3e-2)


@pytest.mark.parametrize("n,c,h,cout", [(4, 64, 14, 256), (2, 128, 9, 512), (3, 256, 7, 64)])
def test_bn_relu_conv1x1_matches_fp32_reference(gpu, n, c, h, cout):
    """conv1x1(relu(bn(x))) with BN applied in the GEMM prologue (stats-only BN pass) vs the fp32
    PyTorch composite: output, input/gamma/beta/weight gradients, running statistics."""
    from determined_1_amd.ops.norm import BatchNormAct2d

    torch.manual_seed(n * c + h)
    x = (torch.randn(n, c, h, h, device=gpu) * 1.5 + 0.3).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    bn = BatchNormAct2d(c, relu=True).to(gpu)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    cv = torch.nn.Conv2d(c, cout, 1, bias=False).to(gpu).to(torch.bfloat16).to(memory_format=torch.channels_last)
    dy = torch.randn(n, cout, h, h, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    xf = x.float().detach().requires_grad_(True)
    bnr = torch.nn.BatchNorm2d(c).to(gpu)
    bnr.load_state_dict({k: v for k, v in bn.state_dict().items()})
    wf = cv.weight.float().detach().requires_grad_(True)
    ref = torch.nn.functional.conv2d(torch.relu(bnr(xf)), wf)
    ref.backward(dy.float())

    before = conv.FUSED_COUNTS["bn_relu_conv1x1"]
    xg = x.detach().requires_grad_(True)
    y = conv.bn_relu_conv1x1(xg, bn, cv)
    y.backward(dy)
    assert conv.FUSED_COUNTS["bn_relu_conv1x1"] == before + 1
    tol = dict(rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(y.float(), ref, **tol)
    torch.testing.assert_close(xg.grad.float(), xf.grad, **tol)
    torch.testing.assert_close(cv.weight.grad.float(), wf.grad, rtol=3e-2, atol=3e-2 * (n * h * h) ** 0.5)
    torch.testing.assert_close(bn.weight.grad, bnr.weight.grad, rtol=3e-2, atol=3e-2 * (n * h * h) ** 0.5)
    torch.testing.assert_close(bn.bias.grad, bnr.bias.grad, rtol=3e-2, atol=3e-2 * (n * h * h) ** 0.5)
    torch.testing.assert_close(bn.running_mean, bnr.running_mean, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(bn.running_var, bnr.running_var, rtol=1e-3, atol=1e-3)
    assert int(bn.num_batches_tracked) == 1


@pytest.mark.parametrize("n,h,w", [(2, 224, 224), (3, 37, 50), (1, 8, 9)])
@pytest.mark.parametrize("cin", [3, 4])
@pytest.mark.parametrize("wgrad", ["patch", "gemm", "miopen"])
def test_stem_conv_matches_fp32_reference(gpu, n, h, w, cin, wgrad, monkeypatch):
    """ResNet stem (7x7/2, pad 3, 64 filters) as the det_conv implicit GEMM vs fp32 conv2d: output,
    BN statistics partials of the output, weight gradient (patch kernel, split-M GEMM or MIOpen);
    3-channel input (padded inside) and 4-channel input with a zero 4th channel."""
    monkeypatch.setattr(conv, "STEM_PATCH_WGRAD", wgrad == "patch")
    monkeypatch.setattr(conv, "STEM_NATIVE_WGRAD", wgrad == "gemm")
    before_patch = conv.FUSED_COUNTS["stem_wgrad_patch"]
    torch.manual_seed(n * h + w + cin)
    x3 = torch.randn(n, 3, h, w, device=gpu).to(torch.bfloat16)
    x = x3 if cin == 3 else torch.cat([x3, torch.zeros_like(x3[:, :1])], 1)
    x = x.contiguous(memory_format=torch.channels_last)
    cv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(gpu).to(torch.bfloat16)
    cv = cv.to(memory_format=torch.channels_last)
    before = conv.FUSED_COUNTS["stem"]
    y = conv.stem_conv(x, cv)
    assert conv.FUSED_COUNTS["stem"] == before + 1
    wf = cv.weight.float().detach().requires_grad_(True)
    ref = torch.nn.functional.conv2d(x3.float(), wf, stride=2, padding=3)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    m = y.shape[0] * y.shape[2] * y.shape[3]
    parts = conv.take_partials(y)
    assert parts is not None
    mean, var = _merge(*parts, m)
    yb = y.float().permute(0, 2, 3, 1).reshape(m, 64).double().cpu()
    torch.testing.assert_close(mean, yb.mean(0), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(var, yb.var(0, unbiased=False), rtol=1e-3, atol=1e-4)
    dy = torch.randn_like(ref).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    ref.backward(dy.float())
    torch.testing.assert_close(cv.weight.grad.float(), wf.grad, rtol=2e-2, atol=2e-3 * m ** 0.5)
    assert conv.FUSED_COUNTS["stem_wgrad_patch"] == before_patch + (1 if wgrad == "patch" else 0)


@pytest.mark.parametrize("n,h,w", [(2, 224, 224), (3, 37, 50), (1, 8, 9)])
def test_stem_patch_wgrad_exact_on_integer_operands(gpu, n, h, w):
    """det_stemp_wgrad (dY and the chunk's input rows staged once; 4-channel pixels read as the
    8-byte rows of transposed fragment reads) == conv2d_weight exactly on small integers."""
    from determined_1_amd.ops import _lib

    g = torch.Generator(device="cpu").manual_seed(n + h + w)
    x = torch.randint(-2, 3, (n, 4, h, w), generator=g).to(torch.bfloat16)
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    dy = torch.randint(-2, 3, (n, 64, ho, wo), generator=g).to(torch.bfloat16)
    ref = torch.nn.grad.conv2d_weight(x.float(), (64, 4, 7, 7), dy.float(), stride=2, padding=3)
    lib = _lib.get_lib()
    m = n * ho * wo
    xg = x.to(gpu).contiguous(memory_format=torch.channels_last)
    dyg = dy.to(gpu).contiguous(memory_format=torch.channels_last)
    ws = torch.empty(int(lib.det_stemp_wgrad_ws_elems(m)), dtype=torch.float32, device=gpu)
    out = torch.empty(64, 256, dtype=torch.float32, device=gpu)
    _lib.check(lib.det_stemp_wgrad(torch.cuda.current_stream().cuda_stream, dyg.data_ptr(), xg.data_ptr(),
                                   out.data_ptr(), 0, m, h, w, ho, wo, ws.data_ptr(), 1.0, None, None), "stemp")
    got = conv.unpack_stem_grad(out, 4).cpu()
    torch.testing.assert_close(got, ref, rtol=0, atol=0)
    # ABN: dY staged as the BN-backward apply coef0 * d + coef1 * x + coef2 (small integers and
    # halves: every product and sum exact, so the staged bf16 dY equals the reference apply)
    d = torch.randint(-2, 3, (n, 64, ho, wo), generator=g).to(torch.bfloat16)
    bx = torch.randint(-2, 3, (n, 64, ho, wo), generator=g).to(torch.bfloat16)
    coef = torch.stack([torch.randint(-2, 3, (64,), generator=g).float() / 2,
                        torch.randint(-2, 3, (64,), generator=g).float() / 2,
                        torch.randint(-2, 3, (64,), generator=g).float() / 2])
    dy_apply = (coef[0].view(1, 64, 1, 1) * d.float() + coef[1].view(1, 64, 1, 1) * bx.float()
                + coef[2].view(1, 64, 1, 1)).to(torch.bfloat16)
    ref2 = torch.nn.grad.conv2d_weight(x.float(), (64, 4, 7, 7), dy_apply.float(), stride=2, padding=3)
    dg = d.to(gpu).contiguous(memory_format=torch.channels_last)
    bxg = bx.to(gpu).contiguous(memory_format=torch.channels_last)
    cg = coef.to(gpu).contiguous()
    _lib.check(lib.det_stemp_wgrad(torch.cuda.current_stream().cuda_stream, dg.data_ptr(), xg.data_ptr(),
                                   out.data_ptr(), 0, m, h, w, ho, wo, ws.data_ptr(), 1.0, bxg.data_ptr(),
                                   cg.data_ptr()), "stemp abn")
    torch.testing.assert_close(conv.unpack_stem_grad(out, 4).cpu(), ref2, rtol=0, atol=0)


@pytest.mark.parametrize("n,h,w", [(2, 224, 224), (3, 37, 50), (1, 8, 9), (5, 57, 57), (3, 99, 101)])
def test_stem_patch_fwd_bit_identical_to_gemm(gpu, n, h, w):
    """det_stemp_fwd (the chunk's input rows staged once in LDS, weights resident, persistent
    blocks) == det_stem_conv_fwd (gathering implicit GEMM) bit for bit -- same k order -- including
    chunks that straddle two images; its 256-row statistics partials merge to the output's."""
    from determined_1_amd.ops import _lib

    torch.manual_seed(n + h + w)
    lib = _lib.get_lib()
    x = torch.randn(n, 4, h, w, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = conv.pack_stem_weight((torch.randn(64, 4, 7, 7, device=gpu) * 0.1).to(torch.bfloat16))
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    m = n * ho * wo
    s = torch.cuda.current_stream().cuda_stream
    y0 = torch.empty(m, 64, dtype=torch.bfloat16, device=gpu)
    y1 = torch.full((m, 64), float("nan"), dtype=torch.bfloat16, device=gpu)
    _lib.check(lib.det_stem_conv_fwd(s, x.data_ptr(), wt.data_ptr(), y0.data_ptr(), m, h, w, ho, wo, None, None), "gemm")
    rpb = int(lib.det_stemp_fwd_rows_per_block())
    nrb = (m + rpb - 1) // rpb
    pm = torch.empty(nrb, 64, dtype=torch.float32, device=gpu)
    pq = torch.empty(nrb, 64, dtype=torch.float32, device=gpu)
    _lib.check(lib.det_stemp_fwd(s, x.data_ptr(), wt.data_ptr(), y1.data_ptr(), m, h, w, ho, wo, pm.data_ptr(),
                                 pq.data_ptr()), "stemp_fwd")
    assert torch.equal(y0, y1)
    mean, var = _merge(pm, pq, rpb, m)
    yb = y1.double().cpu()
    torch.testing.assert_close(mean, yb.mean(0), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(var, yb.var(0, unbiased=False), rtol=1e-3, atol=1e-4)


def test_stem_patch_fwd_wide_images_fall_back(gpu):
    """Images too wide for the stem patch: det_stemp_fwd declines (-6) and stem_conv takes the
    gathering GEMM."""
    from determined_1_amd.ops import _lib

    x = torch.randn(1, 3, 9, 480, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    cv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(gpu).to(torch.bfloat16)
    lib = _lib.get_lib()
    x4 = conv.pad_channels4(x)
    wt = conv.pack_stem_weight(cv.weight)
    y = torch.empty(5 * 240, 64, dtype=torch.bfloat16, device=gpu)
    assert lib.det_stemp_fwd(torch.cuda.current_stream().cuda_stream, x4.data_ptr(), wt.data_ptr(), y.data_ptr(),
                             5 * 240, 9, 480, 5, 240, None, None) == -6
    # 225 x 225: a 256-pixel chunk that straddles two images spans 17 padded rows of 231 pixels
    x2 = torch.zeros(2, 4, 225, 225, device=gpu, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y2 = torch.empty(2 * 113 * 113, 64, dtype=torch.bfloat16, device=gpu)
    assert lib.det_stemp_fwd(torch.cuda.current_stream().cuda_stream, x2.data_ptr(), wt.data_ptr(), y2.data_ptr(),
                             2 * 113 * 113, 225, 225, 113, 113, None, None) == -6
    before = dict(conv.STEM_FWD_COUNTS)
    out = conv.stem_conv(x, cv)
    assert conv.STEM_FWD_COUNTS["gemm"] == before["gemm"] + 1
    ref = torch.nn.functional.conv2d(x.float(), cv.weight.float(), stride=2, padding=3)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)


def test_u8_normalize_pad4(gpu):
    from determined_1_amd.ops.functional import u8_normalize

    g = torch.Generator().manual_seed(0)
    u8 = torch.randint(0, 256, (3, 17, 19, 3), generator=g, dtype=torch.uint8)
    mean, std = (0.485 * 255, 0.456 * 255, 0.406 * 255), (0.229 * 255, 0.224 * 255, 0.225 * 255)
    ref = u8_normalize(u8, mean, std, out_dtype=torch.bfloat16, pad4=True)
    got = u8_normalize(u8.to(gpu), mean, std, out_dtype=torch.bfloat16, pad4=True)
    assert got.shape == (3, 4, 17, 19) and got.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(got.cpu().float(), ref.float(), rtol=1e-2, atol=1e-2)
    assert float(got[:, 3].abs().max()) == 0.0


def test_u8_normalize_pad4_quad_kernel_bit_equal(gpu):
    """The four-pixel C=3 kernel (npix % 4 == 0) against the per-pixel kernel (npix % 4 != 0) on the same
    pixels: bit-equal, and within bf16 rounding of the CPU reference."""
    from determined_1_amd.ops.functional import u8_normalize

    g = torch.Generator().manual_seed(1)
    u8 = torch.randint(0, 256, (2, 16, 28, 3), generator=g, dtype=torch.uint8)
    mean, std = (0.485 * 255, 0.456 * 255, 0.406 * 255), (0.229 * 255, 0.224 * 255, 0.225 * 255)
    quad = u8_normalize(u8.to(gpu), mean, std, out_dtype=torch.bfloat16, pad4=True)   # 896 pixels
    part = u8[:, :5, :7].contiguous()                                                 # 70 pixels
    single = u8_normalize(part.to(gpu), mean, std, out_dtype=torch.bfloat16, pad4=True)
    assert torch.equal(quad[:, :, :5, :7], single)
    ref = u8_normalize(u8, mean, std, out_dtype=torch.bfloat16, pad4=True)
    torch.testing.assert_close(quad.cpu().float(), ref.float(), rtol=1e-2, atol=1e-2)
    assert float(quad[:, 3].abs().max()) == 0.0


def test_resnet50_native_stem_matches_miopen(gpu):
    """Three SGD steps of ResNet-50 with the stem on det_conv (4-channel padded input) vs on MIOpen."""
    from determined_1_amd.models import resnet

    def run(native):
        resnet.NATIVE_STEM = native
        torch.manual_seed(0)
        m = resnet.resnet50(num_classes=10).to(gpu).to(memory_format=torch.channels_last).to(torch.bfloat16)
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.float()
        opt = torch.optim.SGD(m.parameters(), lr=0.02, momentum=0.9)
        g = torch.Generator(device="cpu").manual_seed(1)
        x = torch.randn(8, 3, 64, 64, generator=g).to(gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        if native:
            x = conv.pad_channels4(x)
        y = torch.randint(0, 10, (8,), generator=g).to(gpu)
        losses = []
        for _ in range(3):
            opt.zero_grad()
            loss = torch.nn.functional.cross_entropy(m(x).float(), y)
            loss.backward()
            opt.step()
            losses.append(float(loss.detach()))
        return losses

    before = conv.FUSED_COUNTS["stem"]
    ref = run(False)
    got = run(True)
    resnet.NATIVE_STEM = True
    assert conv.FUSED_COUNTS["stem"] - before == 3
    for a, b in zip(got, ref):
        assert abs(a - b) < 0.05 * max(1.0, abs(b)), (got, ref)
