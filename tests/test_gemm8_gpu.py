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


@pytest.mark.parametrize("approx", [False, True])
def test_gemm8_gelu_epilogue_equals_separate_pass(gpu, approx):
    """The fused GELU epilogue writes the same pre-activation and the same activation, bit for bit,
    as the GEMM followed by det_tf_gelu_fwd on its bf16 output."""
    from determined_1_amd.ops import _lib
    from determined_1_amd.ops.gemm8 import gemm8

    torch.manual_seed(3)
    a = torch.randn(700, 768, device=gpu).to(torch.bfloat16)
    w = (torch.randn(3072, 768, device=gpu) * 0.05).to(torch.bfloat16)
    bias = torch.randn(3072, device=gpu).to(torch.bfloat16)
    z = torch.empty(700, 3072, device=gpu, dtype=torch.bfloat16)
    act = torch.empty_like(z)
    gemm8(a, w, bias=bias, out=z, gelu_out=act, gelu=2 if approx else 1)
    z_ref = gemm8(a, w, bias=bias)
    assert torch.equal(z, z_ref)
    sep = torch.empty_like(z)
    _lib.check(_lib.get_lib().det_tf_gelu_fwd(torch.cuda.current_stream().cuda_stream, 1, z.data_ptr(), sep.data_ptr(),
                                              z.numel(), int(approx)), "gelu")
    assert torch.equal(act, sep)
    ref = torch.nn.functional.gelu(z.float(), approximate="tanh" if approx else "none")
    torch.testing.assert_close(act.float(), ref, rtol=1e-2, atol=1e-2)


def test_linear_gelu_routes_large_ffn_to_gemm8(gpu):
    """ops.transformer.linear_gelu at the BERT FFN-in shape runs the fused gemm8 path; forward and
    gradients match the unfused path."""
    from determined_1_amd.ops import transformer as tf

    torch.manual_seed(4)
    x0 = torch.randn(4608, 768, device=gpu).to(torch.bfloat16)
    w0 = (torch.randn(3072, 768, device=gpu) * 0.03).to(torch.bfloat16)
    b0 = (torch.randn(3072, device=gpu) * 0.1).to(torch.bfloat16)
    dy = torch.randn(4608, 3072, device=gpu).to(torch.bfloat16)
    res = {}
    for on in (False, True):
        tf.GEMM8_FFN = on
        try:
            x, w, b = (t.clone().requires_grad_(True) for t in (x0, w0, b0))
            before = tf.LINEAR_COUNTS["gemm8_gelu_fwd"]
            y = tf.linear_gelu(x, w, b)
            y.backward(dy)
            assert (tf.LINEAR_COUNTS["gemm8_gelu_fwd"] > before) == on
            res[on] = (y.float(), x.grad.float(), w.grad.float(), b.grad.float())
        finally:
            tf.GEMM8_FFN = False
    for u, v in zip(res[False], res[True]):
        torch.testing.assert_close(v, u, rtol=2e-2, atol=2e-2 * float(u.abs().max()))
