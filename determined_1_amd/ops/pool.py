"""3x3 / stride-2 / pad-1 max pooling and global average pooling for channels_last activations
(``det_pool.hip``).

GPU path: one-byte argmax per output element and a gather backward (no zero fill, no atomics);
CPU tensors and layouts the kernel does not cover (C % 8 != 0, not channels_last, fp16) use
``F.max_pool2d``, which is also the numerics reference of the GPU tests.
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_1_amd.ops import _lib

FALLBACKS = {"count": 0}
LINKED = {"count": 0}  # backward passes that summed a linked shortcut gradient
# the pooled tensor is a fused training BN + ReLU output read by nothing else (the ResNet stem): the
# backward gather applies the ReLU mask and writes that BN's backward partial sums (det_pool.hip
# maxpool_bwd BNB), so the BN backward skips its partial pass over the largest activation
FUSE_BN_BWD = os.environ.get("DET_POOL_BN_BWD", "1") != "0"
BN_BWD_COUNTS = {"fused": 0}
BN_FWD_COUNTS = {"in_pool": 0}  # forwards that applied the producer's deferred BN + ReLU
_DT = {torch.float32: 0, torch.bfloat16: 1}


def _bn_producer(x: torch.Tensor):
    """The fused BN(+ReLU, no residual) node that produced ``x`` when its backward can take its
    partial sums from this pool's backward, else None."""
    from determined_1_amd.ops.norm import _BNActTrain, _observed

    gf = x.grad_fn
    if not (FUSE_BN_BWD and isinstance(gf, _BNActTrain._backward_cls) and getattr(gf, "mask_mode", 0) == 1
            and x.dtype == torch.bfloat16 and not _observed(x)):
        return None
    return gf


def _ok(x: torch.Tensor) -> bool:
    return (x.device.type == "cuda" and x.dim() == 4 and x.dtype in _DT and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last))


class _MaxPool3s2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bn_producer=None, bn_apply=None):
        N, C, H, W = x.shape
        Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty((N, C, Ho, Wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        idx = torch.empty((N, Ho, Wo, C), dtype=torch.uint8, device=x.device)
        st = torch._C._cuda_getCurrentRawStream(x.device.index)
        # bn_apply = (bn_x, scale, shift): x is the unwritten output of the producing BN + ReLU, which
        # the pool applies to each window value itself (ops/conv.py DEFER_AFFINE_APPLY)
        src, sc, sh = (x, None, None) if bn_apply is None else bn_apply
        _lib.check(_lib.get_lib().det_maxpool3s2_fwd(st, _DT[x.dtype], src.data_ptr(), y.data_ptr(), idx.data_ptr(),
                                                     N, H, W, C, None if sc is None else sc.data_ptr(),
                                                     None if sh is None else sh.data_ptr()), "det_maxpool3s2_fwd")
        ctx.save_for_backward(idx)
        ctx.shape = (N, C, H, W)
        ctx.extra_dy = None  # set by a linked shortcut consumer (ops/norm.py linked_conv2d)
        ctx.bn_producer = bn_producer
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
        lib = _lib.get_lib()
        prod, ctx.bn_producer = ctx.bn_producer, None
        bn = [None] * 6
        if prod is not None and getattr(prod, "fused_bwd", None) is None and dy.dtype == torch.bfloat16:
            try:
                xb, _, _, stats = prod.saved_tensors
            except RuntimeError:  # already freed (a second backward)
                xb = None
            if xb is not None and xb.shape == dx.shape and xb.is_contiguous(memory_format=torch.channels_last):
                # partial-sum rows: one per pooled row (row-staged kernel) or per 512 pixels; the
                # BN finalize only sums them (rpb is informational)
                nrb = int(lib.det_maxpool3s2_bwd_partial_rows(N, H, W, C))
                rpb = (N * H * W + nrb - 1) // nrb
                psum = torch.empty(nrb, C, dtype=torch.float32, device=dy.device)
                psumx = torch.empty(nrb, C, dtype=torch.float32, device=dy.device)
                bn = [xb.data_ptr(), stats[0].data_ptr(), stats[2].data_ptr(), stats[3].data_ptr(), psum.data_ptr(),
                      psumx.data_ptr()]
        _lib.check(lib.det_maxpool3s2_bwd(st, _DT[dy.dtype], dy.data_ptr(), None if extra is None else extra.data_ptr(),
                                          idx.data_ptr(), dx.data_ptr(), N, H, W, C, *bn), "det_maxpool3s2_bwd")
        if bn[0] is not None:
            # dx is the masked gradient; the BN backward finalizes these partials (ops/norm.py fused_bwd)
            prod.fused_bwd = (psum, psumx, rpb)
            BN_BWD_COUNTS["fused"] += 1
        return dx, None, None


def max_pool_3x3s2(x: torch.Tensor, bn_exclusive: bool = False) -> torch.Tensor:
    """``F.max_pool2d(x, 3, 2, 1)``.  ``bn_exclusive``: this pool is the only autograd consumer of
    ``x``, the output of a fused BatchNorm+ReLU, whose backward partials can then come from the
    pool's backward (``FUSE_BN_BWD``)."""
    aff = getattr(x, "_det_affine_apply", None)
    if aff is not None and not (bn_exclusive and _ok(x) and aff[3] and x.dtype == torch.bfloat16):
        from determined_1_amd.ops.conv import materialize_fwd_apply

        materialize_fwd_apply(x)  # a deferred BN apply this pool cannot stage
        aff = None
    if _ok(x):
        # (decided here: autograd runs Function.forward with grad mode off)
        prod = _bn_producer(x) if (bn_exclusive and torch.is_grad_enabled()) else None
        if aff is not None:
            x._det_affine_apply = None
            BN_FWD_COUNTS["in_pool"] += 1
        return _MaxPool3s2.apply(x, prod, None if aff is None else aff[:3])
    if x.device.type == "cuda":
        FALLBACKS["count"] += 1
    return F.max_pool2d(x, 3, 2, 1)


class MaxPool3x3s2(nn.Module):
    """Drop-in for ``nn.MaxPool2d(3, stride=2, padding=1)`` (the ResNet stem)."""

    def forward(self, x: torch.Tensor, bn_exclusive: bool = False) -> torch.Tensor:
        return max_pool_3x3s2(x, bn_exclusive)


GAP_COUNTS = {"native": 0}


def _gap_ok(x: torch.Tensor) -> bool:
    return (x.device.type == "cuda" and x.dim() == 4 and x.dtype in _DT and x.shape[1] % 256 == 0
            and x.is_contiguous(memory_format=torch.channels_last))


class _GlobalAvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        y = torch.empty((N, C), dtype=x.dtype, device=x.device)
        st = torch._C._cuda_getCurrentRawStream(x.device.index)
        _lib.check(_lib.get_lib().det_gap_fwd(st, _DT[x.dtype], x.data_ptr(), y.data_ptr(), N, H * W, C), "det_gap_fwd")
        ctx.shape = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W = ctx.shape
        dy = dy.contiguous()
        dx = torch.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        st = torch._C._cuda_getCurrentRawStream(dy.device.index)
        _lib.check(_lib.get_lib().det_gap_bwd(st, _DT[dy.dtype], dy.data_ptr(), dx.data_ptr(), N, H * W, C),
                   "det_gap_bwd")
        return dx


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """``torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)`` (the ResNet head) for channels_last
    activations with C % 256 == 0 on ``det_pool.hip`` (``det_gap_fwd`` / ``det_gap_bwd``); other
    inputs take the torch path, which is also the numerics reference of the GPU test."""
    if getattr(x, "_det_affine_apply", None) is not None:
        from determined_1_amd.ops.conv import materialize_fwd_apply

        materialize_fwd_apply(x)
    if _gap_ok(x):
        GAP_COUNTS["native"] += 1
        return _GlobalAvgPool.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
