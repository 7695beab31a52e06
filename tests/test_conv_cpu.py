"""CPU reference path of the native conv autograd functions (ops/conv.py): the same Python
plumbing the GPU path runs (weight layouts, dgrad through the flipped weight, wgrad into a KRSC
view of channels_last memory), against torch autograd.  The HIP kernels themselves are checked by
tests/test_conv3x3_gpu.py."""
import pytest
import torch
import torch.nn.functional as F

from determined_1_amd.ops import conv


def test_dgrad_weight_layout():
    w = torch.randn(8, 4, 3, 3)
    wd = conv.dgrad_weight(w)
    assert wd.shape == (4, 9 * 8)
    # W'[c][r][s][k] = W[k][c][2-r][2-s]
    v = wd.view(4, 3, 3, 8).float()
    assert torch.equal(v[1, 0, 2, 5], w[5, 1, 2, 0].to(torch.bfloat16).float())


@pytest.mark.parametrize("stride", [1, 2])
def test_conv_rs_function_cpu_reference(stride):
    torch.manual_seed(0)
    x = torch.randn(2, 16, 9, 9, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.nn.Parameter((torch.randn(32, 16, 3, 3) * 0.1).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last))
    xr = x.float().requires_grad_(True)
    x.requires_grad_(True)
    y = conv._ConvRS.apply(x, w, stride, 1, False)
    dy = torch.randn_like(y.float()).to(torch.bfloat16)
    y.backward(dy)
    wr = w.detach().float().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=stride, padding=1)
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, rtol=2e-2, atol=5e-2)


def test_conv_wgrad_cpu_matches_autograd():
    torch.manual_seed(1)
    x = torch.randn(2, 8, 7, 7)
    dy = torch.randn(2, 4, 4, 4)
    out = torch.empty(4, 9 * 8)
    conv.conv_wgrad(dy, x, out, 3, 3, 2, 1)
    ref = torch.nn.grad.conv2d_weight(x, (4, 8, 3, 3), dy, stride=2, padding=1)
    torch.testing.assert_close(out.view(4, 3, 3, 8).permute(0, 3, 1, 2), ref)
