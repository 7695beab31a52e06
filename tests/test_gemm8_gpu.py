"""det_gemm8 (ops/csrc/det_gemm8.hip): the eight-phase 256 x 256 GEMM against an fp32 PyTorch
reference, both staging schedules, ragged M / N edges, bias in fp32 and bf16, strided rows, and
repeated launches (a schedule race shows up as launch-to-launch differences)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(a, b, bias=None):
    c = a.float() @ b.float().t()
    if bias is not None:
        c = c + bias.float()
    return c


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (512, 768, 768), (4608, 2304, 768), (300, 264, 128),
                                   (1000, 3072, 192), (4608, 768, 3072), (77, 8, 64)])
def test_gemm8_matches_fp32_reference(gpu, mode, m, n, k):
    from determined_1_amd.ops.gemm8 import gemm8

    torch.manual_seed(m + n + k)
    a = torch.randn(m, k, device=gpu).to(torch.bfloat16)
    b = torch.randn(n, k, device=gpu).to(torch.bfloat16)
    c = gemm8(a, b, mode=mode)
    ref = _ref(a, b)
    torch.testing.assert_close(c.float(), ref, rtol=1e-2, atol=1e-2 * k ** 0.5)
    # bit-exact vs itself across launches: no schedule race
    for _ in range(3):
        assert torch.equal(gemm8(a, b, mode=mode), c)


@pytest.mark.parametrize("bias_dtype", [torch.float32, torch.bfloat16])
def test_gemm8_bias_and_strided_rows(gpu, bias_dtype):
    from determined_1_amd.ops.gemm8 import gemm8

    torch.manual_seed(0)
    big = torch.randn(600, 640, device=gpu).to(torch.bfloat16)
    a = big[:, :512]  # row stride 640
    b = torch.randn(392, 512, device=gpu).to(torch.bfloat16)
    bias = torch.randn(392, device=gpu).to(bias_dtype)
    out = torch.empty(600, 400, device=gpu, dtype=torch.bfloat16)[:, :392]
    c = gemm8(a, b, bias=bias, out=out)
    torch.testing.assert_close(c.float(), _ref(a, b, bias), rtol=1e-2, atol=0.25)


def test_gemm8_rejects_unsupported(gpu):
    from determined_1_amd.ops.gemm8 import gemm8, supported

    a = torch.randn(64, 96, device=gpu).to(torch.bfloat16)
    b = torch.randn(64, 96, device=gpu).to(torch.bfloat16)
    assert not supported(a, b)
    with pytest.raises(ValueError):
        gemm8(a, b)
