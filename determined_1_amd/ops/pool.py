"""3x3 / stride-2 / pad-1 max pooling for channels_last activations (``det_pool.hip``).

GPU path: one-byte argmax per output element and a gather backward (no zero fill, no atomics);
CPU tensors and layouts the kernel does not cover (C % 8 != 0, not channels_last, fp16) use
``F.max_pool2d``, which is also the numerics reference of the GPU tests.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_1_amd.ops import _lib

FALLBACKS = {"count": 0}
LINKED = {"count": 0}  # backward passes that summed a linked shortcut gradient
_DT = {torch.float32: 0, torch.bfloat16: 1}


def _ok(x: torch.Tensor) -> bool:
    return (x.device.type == "cuda" and x.dim() == 4 and x.dtype in _DT and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last))


class _MaxPool3s2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty((N, C, Ho, Wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        idx = torch.empty((N, Ho, Wo, C), dtype=torch.uint8, device=x.device)
        st = torch._C._cuda_getCurrentRawStream(x.device.index)
        _lib.check(_lib.get_lib().det_maxpool3s2_fwd(st, _DT[x.dtype], x.data_ptr(), y.data_ptr(), idx.data_ptr(),
                                                     N, H, W, C), "det_maxpool3s2_fwd")
        ctx.save_for_backward(idx)
        ctx.shape = (N, C, H, W)
        ctx.extra_dy = None  # set by a linked shortcut consumer (ops/norm.py linked_conv2d)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, C, H, W = ctx.shape
        dy = dy.contiguous(memory_format=torch.channels_last)
        # a linked projection shortcut of the pooled output (ops/norm.py linked_conv2d, ResNet layer1)
        # handed its input gradient here instead of to autograd: summed in the gather kernel
        extra, ctx.extra_dy = getattr(ctx, "extra_dy", None), None
        if extra is not None:
            if not isinstance(extra, torch.Tensor):
                from determined_1_amd.ops.conv import full_res_grad

                extra = full_res_grad(extra)
            extra = extra.to(dy.dtype).contiguous(memory_format=torch.channels_last)
            if extra.shape != dy.shape:
                raise RuntimeError(f"linked max-pool gradient shape {tuple(extra.shape)} != {tuple(dy.shape)}")
            LINKED["count"] += 1
        dx = torch.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        st = torch._C._cuda_getCurrentRawStream(dy.device.index)
        _lib.check(_lib.get_lib().det_maxpool3s2_bwd(st, _DT[dy.dtype], dy.data_ptr(),
                                                     None if extra is None else extra.data_ptr(), idx.data_ptr(),
                                                     dx.data_ptr(), N, H, W, C), "det_maxpool3s2_bwd")
        return dx


def max_pool_3x3s2(x: torch.Tensor) -> torch.Tensor:
    """``F.max_pool2d(x, 3, 2, 1)``."""
    if _ok(x):
        return _MaxPool3s2.apply(x)
    if x.device.type == "cuda":
        FALLBACKS["count"] += 1
    return F.max_pool2d(x, 3, 2, 1)


class MaxPool3x3s2(nn.Module):
    """Drop-in for ``nn.MaxPool2d(3, stride=2, padding=1)`` (the ResNet stem)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return max_pool_3x3s2(x)
