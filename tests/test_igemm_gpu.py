"""Numerics of the pipelined implicit-GEMM convolution (ops/csrc/det_igemm.hip) against plain
PyTorch fp32 references: 1x1 and 3x3 convs at stride 1/2 with padding and ragged row tails, the
fused BatchNorm statistics, and the stride-1 input gradients expressed as forward convs."""
import pytest
import torch
import torch.nn.functional as F

from determined_1_amd.ops import conv

pytestmark = pytest.mark.gpu

CASES = [  # (Nb, Cin, H, W, Cout, R, stride, pad)
    (2, 64, 14, 14, 64, 3, 1, 1),
    (3, 128, 7, 9, 128, 3, 1, 1),     # ragged: M = 189
    (2, 128, 15, 15, 256, 3, 2, 1),   # stride 2, odd input
    (4, 256, 28, 28, 128, 3, 1, 1),   # M = 3136: several 256-row blocks + tail
    (3, 256, 5, 7, 64, 1, 1, 0),      # dense 1x1
    (2, 512, 14, 14, 1024, 1, 2, 0),  # 1x1 stride-2 gather
    (1, 64, 56, 56, 256, 1, 1, 0),
]


def _data(case, gpu, seed=0):
    nb, cin, h, w, cout, r, st, pad = case
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(nb, cin, h, w, generator=g).to(torch.bfloat16)
    wt = (torch.randn(cout, cin, r, r, generator=g) / (cin * r * r) ** 0.5).to(torch.bfloat16)
    xg = x.to(gpu).contiguous(memory_format=torch.channels_last)
    wg = wt.to(gpu).contiguous(memory_format=torch.channels_last)
    return x, wt, xg, wg


@pytest.mark.parametrize("case", CASES)
def test_igemm_forward_matches_conv2d(gpu, case):
    nb, cin, h, w, cout, r, st, pad = case
    x, wt, xg, wg = _data(case, gpu)
    y, _ = conv.igemm_conv(xg, wg, stride=st, pad=pad)
    ref = F.conv2d(x.float(), wt.float(), stride=st, padding=pad)
    assert y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float().cpu(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("case", [CASES[1], CASES[3], CASES[5]])
def test_igemm_stats(gpu, case):
    nb, cin, h, w, cout, r, st, pad = case
    x, wt, xg, wg = _data(case, gpu, seed=1)
    y, (pm, pq, rpb) = conv.igemm_conv(xg, wg, stride=st, pad=pad, stats=True)
    yr = y.permute(0, 2, 3, 1).reshape(-1, cout).double().cpu()
    m = yr.shape[0]
    nrb = pm.shape[0]
    assert nrb == (m + rpb - 1) // rpb
    cnt = torch.full((nrb, 1), float(rpb), dtype=torch.float64)
    cnt[-1, 0] = float(m - (nrb - 1) * rpb)
    pmd, pqd = pm.double().cpu(), pq.double().cpu()
    mean = (pmd * cnt).sum(0) / m
    var = (pqd + cnt * (pmd - mean) ** 2).sum(0) / m
    torch.testing.assert_close(mean, yr.mean(0), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(var, yr.var(0, unbiased=False), rtol=1e-4, atol=1e-5)


def test_igemm_exact_integer_operands(gpu):
    """Small integers (exact in bf16 and fp32): any tap / channel / row mix-up shows exactly."""
    nb, cin, h, w, cout = 2, 64, 9, 11, 128
    x = torch.randint(-2, 3, (nb, cin, h, w)).to(torch.bfloat16)
    wt = torch.randint(-2, 3, (cout, cin, 3, 3)).to(torch.bfloat16)
    y, _ = conv.igemm_conv(x.to(gpu).contiguous(memory_format=torch.channels_last),
                           wt.to(gpu).contiguous(memory_format=torch.channels_last), stride=1, pad=1)
    ref = F.conv2d(x.float(), wt.float(), padding=1)
    assert torch.equal(y.float().cpu(), ref)


@pytest.mark.parametrize("cin,cout,r", [(64, 64, 3), (128, 256, 3), (256, 64, 1)])
def test_igemm_dgrad_as_forward_conv(gpu, cin, cout, r):
    """Stride-1 input gradient = forward conv of dY against the flipped, transposed weight."""
    nb, h, w = 2, 10, 12
    pad = r // 2
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(nb, cin, h, w, generator=g, requires_grad=True)
    wt = (torch.randn(cout, cin, r, r, generator=g) / (cin * r * r) ** 0.5).to(torch.bfloat16).float()
    dy = torch.randn(nb, cout, h, w, generator=g).to(torch.bfloat16).float()
    F.conv2d(x, wt, padding=pad).backward(dy)
    wflip = wt.flip(2, 3).transpose(0, 1).contiguous()  # [cin, cout, r, r]
    dx, _ = conv.igemm_conv(dy.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last),
                            wflip.to(gpu, torch.bfloat16).contiguous(memory_format=torch.channels_last), stride=1, pad=pad)
    torch.testing.assert_close(dx.float().cpu(), x.grad, rtol=2e-2, atol=2e-2)
