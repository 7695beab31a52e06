"""``det_gemm8`` (ops/csrc/det_gemm8.hip): C = A . B^T (+ bias) for bf16 K-contiguous operands on a
256 x 256 tile with an eight-phase ping-pong schedule (LDS-DMA staging, counted vmcnt, raw
barriers).  Used for the large BERT Linear passes (ops/transformer.py) where it is measured faster
than the vendor BLAS; ``scripts/bench_gemm8.py`` times it against torch.mm per shape."""
from typing import Optional

import torch

from determined_1_amd.ops import _lib
from determined_1_amd.ops._lib import get_lib

MODE = 1  # staging schedule (det_gemm8.hip header): 1 paired, 0 balanced


def supported(a: torch.Tensor, b: torch.Tensor) -> bool:
    """a [M, K], b [N, K]: bf16 CUDA tensors with unit K stride, K % 64 == 0, N % 8 == 0."""
    return (a.is_cuda and b.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2
            and b.dim() == 2 and a.shape[1] == b.shape[1] and a.shape[1] % 64 == 0 and b.shape[0] % 8 == 0
            and a.stride(1) == 1 and b.stride(1) == 1 and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0
            and ((a.shape[0] - 1) * a.stride(0) + a.shape[1]) * 2 < (1 << 31)
            and ((b.shape[0] - 1) * b.stride(0) + b.shape[1]) * 2 < (1 << 31))


def gemm8(a: torch.Tensor, b: torch.Tensor, bias: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
          mode: Optional[int] = None, gelu_out: Optional[torch.Tensor] = None, gelu: int = 0) -> torch.Tensor:
    """a [M, K] @ b[N, K]^T (+ bias[N]) -> bf16 [M, N].  gelu 1 (erf) / 2 (tanh): also writes
    gelu(result) into ``gelu_out`` (same shape and strides as the result).  Raises if the shape is not
    supported."""
    if not supported(a, b):
        raise ValueError(f"gemm8: unsupported operands {tuple(a.shape)} {a.dtype} / {tuple(b.shape)} {b.dtype}")
    m, k = a.shape
    n = b.shape[0]
    if out is None:
        out = torch.empty(m, n, dtype=torch.bfloat16, device=a.device)
    assert out.dtype == torch.bfloat16 and out.stride(1) == 1 and out.stride(0) % 8 == 0 and out.data_ptr() % 16 == 0
    bias_dt = 0
    if bias is not None:
        assert bias.is_contiguous() and bias.numel() == n
        bias_dt = 1 if bias.dtype == torch.float32 else 2
        assert bias.dtype in (torch.float32, torch.bfloat16)
    if gelu:
        assert gelu_out is not None and gelu_out.shape == out.shape and gelu_out.stride() == out.stride()
        assert gelu_out.dtype == torch.bfloat16 and gelu_out.data_ptr() % 16 == 0
    st = torch.cuda.current_stream(a.device).cuda_stream
    _lib.check(get_lib().det_gemm8(st, a.data_ptr(), b.data_ptr(), out.data_ptr(),
                                   bias.data_ptr() if bias is not None else None, bias_dt, m, n, k,
                                   a.stride(0), b.stride(0), out.stride(0), MODE if mode is None else mode,
                                   gelu_out.data_ptr() if gelu else None, int(gelu)), "gemm8")
    return out
