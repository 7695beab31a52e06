"""BatchNorm-backward fusion into the 1x1 input-gradient GEMM (det_conv_nt_bnbwd +
det_bn_bwd_from_partials): the epilogue's masked gradient and partial sums against an fp32
PyTorch composite for both mask modes (ReLU recomputed from x / forward mask bits with the
identity-shortcut gradient summed in), and ResNet-50 gradients with the fusion on vs off."""
import pytest
import torch

from determined_1_amd.ops import _lib, conv

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("m,c,k", [(1000, 128, 256), (4096, 64, 64), (777, 256, 512)])
def test_bnbwd_epilogue_matches_composite(gpu, mode, m, c, k):
    g = torch.Generator(device="cpu").manual_seed(m + c + mode)
    dy = torch.randn(m, k, generator=g).to(torch.bfloat16)
    w = (torch.randn(c, k, generator=g) / k ** 0.5).to(torch.bfloat16)  # B operand = the transposed conv weight
    x = torch.randn(m, c, generator=g).to(torch.bfloat16)
    mean = torch.randn(c, generator=g) * 0.1
    scale = torch.rand(c, generator=g) + 0.5
    shift = torch.randn(c, generator=g) * 0.2
    add = torch.randn(m, c, generator=g).to(torch.bfloat16) if mode == 2 else None
    pre = x.float() * scale + shift + (torch.randn(m, c, generator=g) if mode == 2 else 0.0)
    mask = pre > 0
    bits = None
    if mode == 2:
        mb = mask.reshape(-1, 8).to(torch.int32)
        bits = (mb * (2 ** torch.arange(8, dtype=torch.int32))).sum(1).to(torch.uint8)
    # reference: dX = dY . W (W is the [c, k] transposed-weight GEMM operand: C = A . B^T with B [c, k])
    dxr = (dy.float() @ w.float().t()).to(torch.bfloat16).float()
    if mode == 2:
        dxr = dxr + add.float()
    d_ref = torch.where(mask, dxr, torch.zeros_like(dxr)).to(torch.bfloat16).float()
    rpb = conv.rows_per_block(c)
    nrb = (m + rpb - 1) // rpb
    psum = torch.empty(nrb, c, device=gpu)
    psumx = torch.empty(nrb, c, device=gpu)
    d = torch.empty(m, c, dtype=torch.bfloat16, device=gpu)
    dev = lambda t: None if t is None else t.to(gpu).contiguous()  # noqa: E731
    dyg, wg, xg, meang, scg, shg, addg, bitsg = (dev(t) for t in (dy, w, x, mean, scale, shift, add, bits))
    _lib.check(_lib.get_lib().det_conv_nt_bnbwd(
        torch.cuda.current_stream().cuda_stream, dyg.data_ptr(), wg.data_ptr(), d.data_ptr(), m, c, k,
        xg.data_ptr(), meang.data_ptr(), scg.data_ptr(), shg.data_ptr(), None if bitsg is None else bitsg.data_ptr(),
        None if addg is None else addg.data_ptr(), psum.data_ptr(), psumx.data_ptr(), mode), "bnbwd")
    torch.cuda.synchronize()
    got = d.float().cpu()
    # one bf16 rounding of the accumulated product may differ by an ulp from torch's rounding
    torch.testing.assert_close(got, d_ref, rtol=2e-2, atol=2e-2)
    assert torch.equal(got == 0, d_ref == 0) or (got[(got == 0) != (d_ref == 0)].abs().max() < 1e-2)
    s_ref = got.double().sum(0)
    sx_ref = (got.double() * (x.double() - mean.double())).sum(0)
    torch.testing.assert_close(psum.double().sum(0).cpu(), s_ref, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(psumx.double().sum(0).cpu(), sx_ref, rtol=1e-4, atol=1e-3)


def test_resnet50_grads_with_and_without_bn_bwd_fusion(gpu):
    """One backward of ResNet-50 (bf16, fused BN, native convs) from identical weights and data:
    every parameter gradient with the fusion matches the unfused path."""
    from determined_1_amd.models import resnet

    def run(fuse):
        conv.FUSE_BN_BWD = fuse
        torch.manual_seed(0)
        m = resnet.resnet50(num_classes=10, zero_init_residual=False).to(gpu).to(
            memory_format=torch.channels_last).to(torch.bfloat16)
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.float()
        g = torch.Generator(device="cpu").manual_seed(1)
        x = torch.randn(4, 3, 64, 64, generator=g).to(gpu).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = torch.randint(0, 10, (4,), generator=g).to(gpu)
        loss = torch.nn.functional.cross_entropy(m(conv.pad_channels4(x)).float(), y)
        loss.backward()
        return {n: p.grad.float().clone() for n, p in m.named_parameters()}

    before = dict(conv.BN_BWD_COUNTS)
    ref = run(False)
    got = run(True)
    conv.FUSE_BN_BWD = True
    fused = conv.BN_BWD_COUNTS["fused"] - before["fused"]
    assert fused >= 16 + 12  # bn2 -> conv3 in all 16 blocks, block outputs -> next conv1 (>= 12 identity links)
    for n in ref:
        a, b = got[n], ref[n]
        scale = float(b.abs().max()) + 1e-6
        assert float((a - b).abs().max()) <= 0.05 * scale, (n, float((a - b).abs().max()), scale)
