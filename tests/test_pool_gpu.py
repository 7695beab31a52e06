"""ResNet-stem max pooling (ops/csrc/det_pool.hip) vs torch's fp32 max_pool2d on CPU."""
import pytest
import torch
import torch.nn.functional as F

from determined_1_amd.ops import pool

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["gather", "rows"])
def fwd_kernel(request):
    """Both max-pool forwards: the per-output gather (default) and the row-staged one."""
    from determined_1_amd.ops import _lib

    lib = _lib.get_lib()
    lib.det_maxpool3s2_set_fwd_rows(1 if request.param == "rows" else 0)
    yield request.param
    lib.det_maxpool3s2_set_fwd_rows(0)


@pytest.mark.parametrize("N,C,H,W,dt", [(4, 64, 112, 112, torch.bfloat16), (2, 16, 15, 9, torch.float32),
                                        (3, 8, 8, 8, torch.bfloat16), (1, 32, 1, 5, torch.float32)])
def test_maxpool3s2_matches_torch(gpu, fwd_kernel, N, C, H, W, dt):
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W).to(dt).float()  # bf16 values: ties inside windows do occur
    dy_shape = F.max_pool2d(x, 3, 2, 1).shape
    dy = torch.randn(dy_shape).to(dt).float()
    ref_in = x.clone().requires_grad_(True)
    ref = F.max_pool2d(ref_in, 3, 2, 1)
    ref.backward(dy)
    dut_in = x.to(gpu, dt).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    before = pool.FALLBACKS["count"]
    out = pool.max_pool_3x3s2(dut_in)
    assert pool.FALLBACKS["count"] == before, "fell back to torch"
    assert out.is_contiguous(memory_format=torch.channels_last)
    out.backward(dy.to(gpu, dt).contiguous(memory_format=torch.channels_last))
    torch.testing.assert_close(out.float().cpu(), ref.detach(), atol=0, rtol=0)
    # fp32: up to 4 overlapping windows summed in a different order than torch's scatter
    tol = dict(atol=1e-6, rtol=1e-5) if dt == torch.float32 else dict(atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(dut_in.grad.float().cpu(), ref_in.grad, **tol)


@pytest.mark.parametrize("native_shortcut", [True, False])
def test_maxpool_linked_projection_gradient(gpu, native_shortcut, monkeypatch):
    """ResNet layer1: the pooled stem output feeds conv1 and a stride-1 projection shortcut; the
    shortcut's input gradient is linked to the pool's backward (ops/norm.py linked_conv2d) and summed
    in its gather kernel.  Checked against the fp32 CPU composite with autograd's add."""
    from determined_1_amd.ops import conv as convops
    from determined_1_amd.ops import norm

    monkeypatch.setattr(norm, "MAXPOOL_LINK", True)
    torch.manual_seed(0)
    N, C, H, W, Co = 8, 64, 56, 56, 256
    x = torch.randn(N, C, H, W).to(torch.bfloat16).float()
    w1 = (torch.randn(64, C, 1, 1) / C ** 0.5).to(torch.bfloat16)
    ws = (torch.randn(Co, C, 1, 1) / C ** 0.5).to(torch.bfloat16)
    g1 = torch.randn(N, 64, H // 2, W // 2).to(torch.bfloat16)
    gs = torch.randn(N, Co, H // 2, W // 2).to(torch.bfloat16)

    ref_in = x.clone().requires_grad_(True)
    p = F.max_pool2d(ref_in, 3, 2, 1)
    ((F.conv2d(p, w1.float()) * g1.float()).sum() + (F.conv2d(p, ws.float()) * gs.float()).sum()).backward()
    ref_x = ref_in.grad

    conv1 = torch.nn.Conv2d(C, 64, 1, bias=False).to(gpu, torch.bfloat16).to(memory_format=torch.channels_last)
    sc = torch.nn.Conv2d(C, Co, 1, bias=False).to(gpu, torch.bfloat16).to(memory_format=torch.channels_last)
    with torch.no_grad():
        conv1.weight.copy_(w1)
        sc.weight.copy_(ws)
    dut_in = x.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    pooled = pool.max_pool_3x3s2(dut_in)
    old = convops.ENABLED
    linked_before = pool.LINKED["count"]
    try:
        if not native_shortcut:
            convops.ENABLED = False  # _LinkedConv (MIOpen conv) path instead of the native shortcut
        ys = norm.linked_conv2d(pooled, sc)
        y1 = conv1(pooled)
        torch.autograd.backward([y1, ys], [g1.to(gpu).contiguous(memory_format=torch.channels_last),
                                           gs.to(gpu).contiguous(memory_format=torch.channels_last)])
    finally:
        convops.ENABLED = old
    assert pool.LINKED["count"] == linked_before + 1, "shortcut gradient was not linked to the pool"
    torch.testing.assert_close(dut_in.grad.float().cpu(), ref_x, atol=5e-2, rtol=2e-2)


@pytest.mark.parametrize("N,C,H,W", [(4, 64, 56, 56), (3, 32, 17, 9)])
def test_maxpool_bn_backward_epilogue(gpu, N, C, H, W, monkeypatch):
    """Stem BN + ReLU -> max-pool with the BN's backward partial sums written by the pool's gather
    (det_pool.hip maxpool_bwd BNB) vs the same GPU chain with the fusion off (the plain gather and
    the BN's own partial pass): the same forward, so the same argmax, and gradients equal up to the
    summation order of the partials.  Also near the fp32 CPU composite, where bf16 rounding of the
    pooled values moves an argmax now and then (a handful of elements)."""
    from determined_1_amd.ops.norm import BatchNormAct2d

    torch.manual_seed(1)
    x = (torch.randn(N, C, H, W) * 2 + 0.3).to(torch.bfloat16).float()
    dy = torch.randn(N, C, (H - 1) // 2 + 1, (W - 1) // 2 + 1).to(torch.bfloat16).float()
    bn = BatchNormAct2d(C, relu=True, fused=True).to(gpu)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C) + 0.5)
        bn.bias.copy_(torch.randn(C) * 0.2)

    def run(fused):
        monkeypatch.setattr(pool, "FUSE_BN_BWD", fused)
        bn.zero_grad(set_to_none=True)
        xin = x.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        before = pool.BN_BWD_COUNTS["fused"]
        out = pool.max_pool_3x3s2(bn(xin), bn_exclusive=True)
        out.backward(dy.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last))
        assert pool.BN_BWD_COUNTS["fused"] == before + int(fused)
        return xin.grad.float().cpu(), bn.weight.grad.cpu(), bn.bias.grad.cpu()

    dx_f, dw_f, db_f = run(True)
    dx_u, dw_u, db_u = run(False)
    torch.testing.assert_close(dw_f, dw_u, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(db_f, db_u, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(dx_f, dx_u, atol=2e-2, rtol=2e-2)

    ref_in = x.clone().requires_grad_(True)
    wr, br = bn.weight.detach().cpu().clone().requires_grad_(True), bn.bias.detach().cpu().clone().requires_grad_(True)
    F.max_pool2d(F.relu(F.batch_norm(ref_in, None, None, wr, br, True)), 3, 2, 1).backward(dy)
    bad = ~torch.isclose(dx_f, ref_in.grad, atol=5e-2, rtol=5e-2)
    assert int(bad.sum()) <= max(8, dx_f.numel() // 2000), int(bad.sum())
    torch.testing.assert_close(dw_f, wr.grad, atol=5e-2, rtol=5e-2)
    torch.testing.assert_close(db_f, br.grad, atol=5e-2, rtol=5e-2)


def test_stem_chain_defers_bn_apply_into_patch_wgrad(gpu):
    """ResNet stem: conv -> BN + ReLU -> pool.  The pool applies the BN + ReLU while reading its
    windows (the activation is never written), its backward writes the BN partials, the BN backward
    only finalizes, and the stem weight gradient stages the BN's backward apply (stemp_wgrad ABN).
    Pooled output bit-equal, weight gradient close to the same chain with the fusions off."""
    from determined_1_amd.models import resnet
    from determined_1_amd.ops import conv as convops

    torch.manual_seed(2)
    img = torch.randn(4, 3, 64, 64)

    def run(fused):
        torch.manual_seed(3)
        m = resnet.resnet50(num_classes=10).to(gpu).to(memory_format=torch.channels_last).to(torch.bfloat16)
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.float()
        old = (pool.FUSE_BN_BWD, convops.DEFER_BN_APPLY, convops.DEFER_AFFINE_APPLY)
        pool.FUSE_BN_BWD = convops.DEFER_BN_APPLY = convops.DEFER_AFFINE_APPLY = fused
        resnet._FWD.depth = 1  # as inside ResNet.forward
        try:
            x = img.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last)
            y = m.maxpool(m.bn1(m._stem(x), defer_affine=True), bn_exclusive=True)
            (y.float() * torch.linspace(-1, 1, y.numel(), device=gpu).view_as(y)).sum().backward()
        finally:
            pool.FUSE_BN_BWD, convops.DEFER_BN_APPLY, convops.DEFER_AFFINE_APPLY = old
            resnet._FWD.depth = 0
        return m.conv1.weight.grad.float().cpu(), m.bn1.weight.grad.cpu(), y.detach().cpu()

    before = (pool.BN_BWD_COUNTS["fused"], convops.BN_APPLY_COUNTS["in_gemm"], pool.BN_FWD_COUNTS["in_pool"])
    wf, gf, yf = run(True)
    assert pool.BN_BWD_COUNTS["fused"] == before[0] + 1
    assert convops.BN_APPLY_COUNTS["in_gemm"] == before[1] + 1, "the stem wgrad did not stage the BN apply"
    assert pool.BN_FWD_COUNTS["in_pool"] == before[2] + 1, "the pool did not apply the stem BN"
    wu, gu, yu = run(False)
    assert torch.equal(yf, yu)  # the pool's BN + ReLU rounds exactly like the materialised apply
    torch.testing.assert_close(wf, wu, atol=2e-2 * float(wu.abs().max()), rtol=2e-2)
    torch.testing.assert_close(gf, gu, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("N,C,H,W", [(8, 2048, 7, 7), (3, 512, 1, 1), (2, 256, 14, 14), (5, 768, 7, 9)])
def test_global_avg_pool_matches_fp32_torch(gpu, N, C, H, W, dt):
    """det_gap_fwd / det_gap_bwd against the fp32 torch head pooling (flatten(adaptive_avg_pool2d))."""
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W, device=gpu).to(dt).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    n0 = pool.GAP_COUNTS["native"]
    y = pool.global_avg_pool(x)
    assert pool.GAP_COUNTS["native"] == n0 + 1  # the HIP path ran, not the torch fallback
    xr = x.detach().float().requires_grad_(True)
    yr = torch.flatten(F.adaptive_avg_pool2d(xr, 1), 1)
    assert y.shape == yr.shape and y.dtype == dt
    tol = 1e-2 if dt == torch.bfloat16 else 1e-5
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
    g = torch.randn(N, C, device=gpu).to(dt)
    (dx,) = torch.autograd.grad(y, x, g)
    (dxr,) = torch.autograd.grad(yr, xr, g.float())
    assert dx.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(dx.float(), dxr, rtol=tol, atol=tol)
    # the gradient is g / HW in fp32 rounded once to dt: bit-exact in bf16, within 1 fp32 ulp in fp32
    # (the device's fp32 division vs torch's)
    exact = (g.float() / (H * W))[:, :, None, None].expand(N, C, H, W).to(dt)
    torch.testing.assert_close(dx, exact, rtol=0 if dt == torch.bfloat16 else 2.4e-7, atol=0)


def test_global_avg_pool_falls_back_off_the_kernel_shapes(gpu):
    x = torch.randn(2, 64, 5, 5, device=gpu).contiguous(memory_format=torch.channels_last)
    n0 = pool.GAP_COUNTS["native"]
    y = pool.global_avg_pool(x)
    assert pool.GAP_COUNTS["native"] == n0
    torch.testing.assert_close(y, x.mean((2, 3)))
