"""ResNet-stem max pooling (ops/csrc/det_pool.hip) vs torch's fp32 max_pool2d on CPU."""
import pytest
import torch
import torch.nn.functional as F

from determined_1_amd.ops import pool

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,C,H,W,dt", [(4, 64, 112, 112, torch.bfloat16), (2, 16, 15, 9, torch.float32),
                                        (3, 8, 8, 8, torch.bfloat16), (1, 32, 1, 5, torch.float32)])
def test_maxpool3s2_matches_torch(gpu, N, C, H, W, dt):
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
