"""Fused training BatchNorm (+ residual add) (+ ReLU) for channels_last activations.

GPU path: ``det_norm.hip`` (3 launches forward, 3 backward; see the header of that file for the
byte accounting).  CPU path: the plain PyTorch composite ``relu(batch_norm(x) + residual)``, which
is also the numerics reference the GPU tests compare against.

``BatchNormAct2d`` is a drop-in ``nn.BatchNorm2d`` subclass: same parameters, buffers and
state-dict keys (so checkpoints stay interchangeable with stock torchvision-style models), with
``forward(x, residual=None)`` applying ``act(bn(x) + residual)`` in one fused pass.

Layouts the kernels do not cover (C % 8 != 0, non-channels_last GPU tensors, fp16) take the
composite path and are counted in ``FALLBACKS`` so a benchmark can assert it stayed native.
"""
from typing import Optional, Tuple

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_1_amd.ops import _lib
from determined_1_amd.ops import conv as _conv

FALLBACKS = {"count": 0}
SHORTCUT_LINK = os.environ.get("DET_SHORTCUT_LINK", "1") != "0"  # identity-shortcut gradients through the producer's BN backward (A/B switch)
_SYNC_DEBUG = bool(__import__("os").environ.get("DET_SYNC_DEBUG"))


def _dbg(what: str, x: torch.Tensor) -> None:
    if _SYNC_DEBUG:
        torch.cuda.synchronize()
        print(f"[det_norm] {what} ok shape={tuple(x.shape)} dtype={x.dtype}", flush=True)
_DT = {torch.float32: 0, torch.bfloat16: 1}


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _nhwc_ok(x: torch.Tensor) -> bool:
    if x.dtype not in _DT or x.device.type != "cuda":
        return False
    if x.dim() == 4:
        c = x.shape[1]
        return c % 8 == 0 and x.is_contiguous(memory_format=torch.channels_last)
    if x.dim() == 2:
        return x.shape[1] % 8 == 0 and x.is_contiguous()
    return False


def _rows(x: torch.Tensor) -> Tuple[int, int]:
    c = x.shape[1]
    return x.numel() // c, c


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def reference_bn_act(x, residual, weight, bias, running_mean, running_var, training, momentum, eps, relu):
    """The composite the fused kernels implement (fp32 math on CPU)."""
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum if momentum is not None else 0.0, eps)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


class _BNActTrain(torch.autograd.Function):
    """``act(bn(x) + residual)``.  ``link`` (identity shortcuts): the residual is the output of
    another ``_BNActTrain`` (the previous block's) that also feeds this block's first conv; its
    gradient is then handed to that producer's backward as a second upstream gradient (``dy2``,
    summed inside the BN-backward kernels) instead of returned to autograd, which would add it to
    the conv's input gradient with a separate elementwise pass over the whole activation."""

    @staticmethod
    def forward(ctx, x, residual, weight, bias, running_mean, running_var, nbt, momentum, eps, relu, link=None,
                defer=False, res_affine=None, defer_affine=False):
        M, C = _rows(x)
        lib = _lib.get_lib()
        fmt = torch.channels_last if x.dim() == 4 else torch.contiguous_format
        y = torch.empty_like(x, memory_format=fmt)
        stats = torch.empty((4, C), dtype=torch.float32, device=x.device)
        if residual is not None:
            residual = residual.to(x.dtype).contiguous(memory_format=fmt)
        mbits = torch.empty(x.numel() // 8, dtype=torch.uint8, device=x.device) \
            if (relu and residual is not None) else None
        from determined_1_amd.ops.conv import take_partials

        parts = take_partials(x)  # statistics already computed by the producing GEMM's epilogue
        ws = torch.empty(int(lib.det_bn_fin_ws_elems(C) if parts is not None else lib.det_bn_ws_elems(M, C)),
                         dtype=torch.float32, device=x.device)
        defer = bool(defer and parts is not None and relu and residual is not None and mbits is not None
                     and x.dtype == torch.bfloat16 and fmt == torch.channels_last)
        # res_affine = (r, scale, shift): the residual is a BN output whose apply was deferred (the
        # projection shortcut's, below); this apply computes it from r (det_norm.hip RES 2)
        if res_affine is not None and not (parts is not None and relu and x.dtype == torch.bfloat16):
            _conv.materialize_affine_apply(residual, res_affine)
            res_affine = None
        res_src, rs, rh = (residual, None, None) if res_affine is None else res_affine
        # defer_affine: a BN without residual whose only consumer applies it itself -- a residual BN
        # apply taking res_affine (ResNet's projection-shortcut BN, no ReLU) or the max-pool forward
        # (the stem BN + ReLU): finalize only, the output stays unwritten
        defer_affine = bool(defer_affine and parts is not None and residual is None
                            and x.dtype == torch.bfloat16 and fmt == torch.channels_last)
        if parts is not None:
            pm, pq, rpb = parts
            _lib.check(
                lib.det_bn_fwd_from_partials(
                    _stream(x), _DT[x.dtype], x.data_ptr(), _ptr(res_src), y.data_ptr(), M, C, int(rpb),
                    int(pm.shape[0]), pm.data_ptr(), pq.data_ptr(),
                    _ptr(weight), _ptr(bias), _ptr(running_mean), _ptr(running_var), _ptr(nbt),
                    float(-1.0 if momentum is None else momentum), float(eps), int(bool(relu)),
                    0 if (defer or defer_affine) else 1,
                    stats[0].data_ptr(), stats[1].data_ptr(), stats[2].data_ptr(), stats[3].data_ptr(), _ptr(mbits),
                    ws.data_ptr(), _ptr(rs), _ptr(rh),
                ),
                "bn_fwd_from_partials",
            )
        else:
            _lib.check(
                lib.det_bn_fwd_train(
                    _stream(x), _DT[x.dtype], x.data_ptr(), _ptr(residual), y.data_ptr(), M, C,
                    _ptr(weight), _ptr(bias), _ptr(running_mean), _ptr(running_var), _ptr(nbt),
                    float(-1.0 if momentum is None else momentum), float(eps), int(bool(relu)),
                    stats[0].data_ptr(), stats[1].data_ptr(), stats[2].data_ptr(), stats[3].data_ptr(),
                    ws.data_ptr(), _ptr(mbits),
                ),
                "bn_fwd_train",
            )
        _dbg("fwd_train", x)
        mask_mode = 0 if not relu else (2 if residual is not None else 1)
        ctx.mask_mode = mask_mode
        ctx.has_res = residual is not None
        ctx.link = link  # producer ctx of the residual (identity shortcut) or None
        if link is not None:
            link.expects_extra = True  # a fused dgrad into the producer must wait for this gradient
        ctx.extra_dy = None  # set by the consumer of this output as identity shortcut
        ctx.fmt = fmt
        ctx.save_for_backward(x, mbits, weight, stats)
        if defer:
            # y stays unwritten: the consuming conv stages (and writes) the apply (ops/conv.py
            # DEFER_FWD_APPLY); bn_act tags the returned tensor
            _DEFERRED["last"] = (y.data_ptr(), (x, res_src, stats[2], stats[3], mbits, rs, rh))
            _conv.FWD_APPLY_COUNTS["deferred"] += 1
        elif defer_affine:
            _DEFERRED["last"] = (y.data_ptr(), ("affine", x, stats[2], stats[3], bool(relu)))
            _conv.AFFINE_APPLY_COUNTS["deferred"] += 1
        if res_affine is not None:
            _conv.AFFINE_APPLY_COUNTS["in_residual"] += 1
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mbits, weight, stats = ctx.saved_tensors
        M, C = _rows(x)
        lib = _lib.get_lib()
        dy = dy.to(x.dtype).contiguous(memory_format=ctx.fmt)
        dy2, ctx.extra_dy = ctx.extra_dy, None
        dy2 = _conv.full_res_grad(dy2)  # a stride-2 projection shortcut's gradient, unfused path
        dx = torch.empty_like(x, memory_format=ctx.fmt)
        want_res = ctx.has_res and (ctx.needs_input_grad[1] or ctx.link is not None)
        dgb = None
        if weight is not None and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3]):
            dgb = torch.empty((2, C), dtype=torch.float32, device=x.device)
        fused, ctx.fused_bwd = getattr(ctx, "fused_bwd", None), None
        if fused is not None:
            # the consuming conv's dgrad epilogue already masked dy (and summed the shortcut
            # gradient into it) and wrote the partial sums: finalize + unmasked apply; the masked
            # gradient is also the residual's gradient (no second tensor)
            assert dy2 is None, "shortcut gradient arrived after the fused dgrad consumed it"
            psum, psumx, rpb = fused
            # [3][C] apply coefficients, then the sliced finalize's scratch
            coef = torch.empty(3 * C + int(lib.det_bn_bwd_scratch_elems(C)), dtype=torch.float32, device=x.device)
            conv_node = x.grad_fn
            if (_conv.DEFER_BN_APPLY and getattr(conv_node, "accepts_bn_apply", False)
                    and getattr(conv_node, "pending_bn_apply", "x") is None and x.dtype == torch.bfloat16
                    and ctx.fmt == torch.channels_last and dy.is_contiguous(memory_format=torch.channels_last)):
                # x came from a native 1x1 conv whose input-gradient GEMM computes dx = A d + B x + C
                # while staging its A operand (ops/conv.py take_pending_apply): finalize only here
                _lib.check(
                    lib.det_bn_bwd_finalize_partials(
                        _stream(x), M, C, _ptr(weight), stats[0].data_ptr(), stats[1].data_ptr(), psum.data_ptr(),
                        psumx.data_ptr(), int(psum.shape[0]), int(rpb), None if dgb is None else dgb[0].data_ptr(),
                        None if dgb is None else dgb[1].data_ptr(), coef.data_ptr(), coef[3 * C:].data_ptr()),
                    "bn_bwd_finalize_partials",
                )
                conv_node.pending_bn_apply = (dx, dy, x, coef)
                _conv.BN_APPLY_COUNTS["deferred"] += 1
                dres = dy if want_res else None
                fused = "deferred"
        if fused is not None and fused != "deferred":
            _lib.check(
                lib.det_bn_bwd_from_partials(
                    _stream(x), _DT[x.dtype], dy.data_ptr(), x.data_ptr(), M, C, _ptr(weight), stats[0].data_ptr(),
                    stats[1].data_ptr(), psum.data_ptr(), psumx.data_ptr(), int(psum.shape[0]), int(rpb),
                    dx.data_ptr(), None if dgb is None else dgb[0].data_ptr(),
                    None if dgb is None else dgb[1].data_ptr(), coef.data_ptr(), coef[3 * C:].data_ptr()),
                "bn_bwd_from_partials",
            )
            dres = dy if want_res else None
        elif fused is None:
            dres = torch.empty_like(x, memory_format=ctx.fmt) if want_res else None
            ws = torch.empty(int(lib.det_bn_ws_elems(M, C)), dtype=torch.float32, device=x.device)
            # an affine BN (no ReLU, no residual: ResNet's projection-shortcut BN) whose input came
            # from a native conv that stages the apply in its input-gradient GEMM: partials and
            # finalize here, the apply there (ops/conv.py take_pending_apply)
            conv_node = x.grad_fn
            defer = (ctx.mask_mode == 0 and dy2 is None and dres is None and _conv.DEFER_BN_APPLY
                     and getattr(conv_node, "accepts_bn_apply", False)
                     and getattr(conv_node, "pending_bn_apply", "x") is None and x.dtype == torch.bfloat16
                     and ctx.fmt == torch.channels_last and dy.is_contiguous(memory_format=torch.channels_last))
            _lib.check(
                lib.det_bn_bwd(
                    _stream(x), _DT[x.dtype], dy.data_ptr(), _ptr(dy2), x.data_ptr(), _ptr(mbits), M, C, ctx.mask_mode,
                    _ptr(weight), stats[0].data_ptr(), stats[1].data_ptr(), stats[2].data_ptr(), stats[3].data_ptr(),
                    dx.data_ptr(), _ptr(dres),
                    None if dgb is None else dgb[0].data_ptr(), None if dgb is None else dgb[1].data_ptr(),
                    ws.data_ptr(), 0 if defer else 1,
                ),
                "bn_bwd",
            )
            if defer:
                off = int(lib.det_bn_bwd_coef_offset(M, C))
                conv_node.pending_bn_apply = (dx, dy, x, ws[off:off + 3 * C])
                _conv.BN_APPLY_COUNTS["deferred"] += 1
        _dbg("bwd", x)
        if ctx.has_res and dres is None and ctx.needs_input_grad[1]:
            raise RuntimeError("residual grad requested but not produced")
        if ctx.link is not None:
            # the producer runs later (its output also feeds our block's first conv, whose input
            # gradient it waits for); it sums dres in its own backward kernels
            hand_linked_grad(ctx.link, dres)
            ctx.link = None
            dres = None
        dw = dgb[0] if dgb is not None and ctx.needs_input_grad[2] else None
        db = dgb[1] if dgb is not None and ctx.needs_input_grad[3] else None
        return dx, dres, dw, db, None, None, None, None, None, None, None, None, None, None


class _LinkedConv(torch.autograd.Function):
    """``conv2d(x, w)`` where ``x`` is the output of a ``_BNActTrain`` that also feeds another conv
    (a ResNet downsample block: ``x`` -> block conv1 and -> shortcut conv).  The input gradient of
    this conv is handed to the producer's backward as its second upstream gradient (summed in the
    BN-backward kernels) instead of returned to autograd, which would add it to the other conv's
    input gradient in a separate elementwise pass over the whole activation.  ``x`` keeps its
    autograd edge (a None gradient is returned), so the producer's backward is ordered after
    this one by the graph itself."""

    @staticmethod
    def forward(ctx, x, weight, stride, padding, dilation, groups, link):
        ctx.save_for_backward(x, weight)
        ctx.conv = (stride, padding, dilation, groups)
        ctx.link = link
        link.expects_extra = True  # a fused dgrad into the producer must wait for this gradient
        return F.conv2d(x, weight, None, stride, padding, dilation, groups)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        stride, padding, dilation, groups = ctx.conv
        dx, dw, _ = torch.ops.aten.convolution_backward(
            dy, x, weight, None, list(stride), list(padding), list(dilation), False, [0] * len(stride), groups,
            [True, bool(ctx.needs_input_grad[1]), False])
        link, ctx.link = ctx.link, None
        if link is None:  # a repeated backward (retain_graph): plain autograd accumulation
            return dx, dw, None, None, None, None, None
        hand_linked_grad(link, dx.contiguous(memory_format=torch.channels_last))
        return None, dw, None, None, None, None, None


def _autocast_keeps(x: torch.Tensor) -> bool:
    """True when autocast (if on) would leave ``x``'s dtype unchanged for a conv."""
    dev = x.device.type
    if not torch.is_autocast_enabled(dev):
        return True
    return torch.get_autocast_dtype(dev) == x.dtype


def _observed(x: torch.Tensor) -> bool:
    """``x``'s own gradient is observable (retain_grad / tensor hooks): the link would hand only
    part of it to autograd, so it must not be used."""
    return bool(x.retains_grad or getattr(x, "_backward_hooks", None))


def hand_linked_grad(link, grad) -> None:
    """Hand ``grad`` (a second upstream gradient of ``link``'s output) to the producer node ``link``,
    whose backward sums it in its own kernels, and check at the end of this backward pass that the
    producer did run and consume it.  It does not when autograd stops at the linked activation
    (``torch.autograd.grad(loss, x)`` / ``backward(inputs=[x])``): the gradient autograd reports for
    ``x`` would then silently lack this consumer's share, so the pass raises instead (and the stale
    gradient is dropped, never summed into a later backward).  ``DET_SHORTCUT_LINK=0`` turns the
    links off for code that needs such partial gradients."""
    if link.extra_dy is not None:
        raise RuntimeError("second upstream gradient linked twice to one producer")
    link.extra_dy = grad

    def check() -> None:
        if getattr(link, "extra_dy", None) is not None:
            link.extra_dy = None
            LINK_COUNTS["unconsumed"] += 1
            raise RuntimeError(
                "a linked shortcut gradient was not consumed: autograd stopped at an activation whose "
                "gradient is summed inside its producer's backward (torch.autograd.grad / backward(inputs=) "
                "on a fused ResNet activation). Set DET_SHORTCUT_LINK=0 to compute such partial gradients.")

    torch.autograd.Variable._execution_engine.queue_callback(check)


LINK_COUNTS = {"unconsumed": 0}


# Link a stride-1 projection of the stem max-pool output (ResNet layer1) to the pool's backward,
# which sums the shortcut's input gradient in its gather kernel (no separate autograd add pass).
# measured on: +0.16 % (3 interleaved pairs, every pair positive; profiles/r4_maxpool_link_ab.jsonl)
MAXPOOL_LINK = os.environ.get("DET_MAXPOOL_LINK", "1") == "1"


def _maxpool_link_ok(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    from determined_1_amd.ops import pool as _pool

    return (MAXPOOL_LINK and isinstance(x.grad_fn, _pool._MaxPool3s2._backward_cls)
            and tuple(conv.stride) == (1, 1) and tuple(conv.padding) == (0, 0) and conv.kernel_size == (1, 1))


def linked_conv2d(x: torch.Tensor, conv: nn.Conv2d) -> torch.Tensor:
    """``conv(x)``; when ``x`` came from the fused BN-act op and feeds another consumer too, the
    conv's input gradient is summed inside the producer's BN-backward kernels (``_LinkedConv``).

    Limitation of the link: autograd sees no gradient for ``x`` from this conv (it is added inside
    the producer's backward), so ``torch.autograd.grad(loss, x)`` taken *without* running the full
    backward would miss this consumer's share.  ``x.retain_grad()`` and ``x.register_hook`` are
    detected and fall back to plain ``conv(x)`` (``_observed``).  1x1 stride-1/2 convs on channels_last
    bf16 take the native path (``ops.conv.shortcut_conv1x1``), with or without the link."""
    _conv.materialize_fwd_apply(x)
    if (SHORTCUT_LINK and conv.bias is None and torch.is_grad_enabled() and x.requires_grad
            and not _observed(x)
            and (isinstance(x.grad_fn, _BNActTrain._backward_cls) or _maxpool_link_ok(x, conv)) and x.dim() == 4
            and x.dtype == conv.weight.dtype and _autocast_keeps(x)
            and x.is_contiguous(memory_format=torch.channels_last) and conv.padding_mode == "zeros"
            and getattr(x.grad_fn, "extra_dy", None) is None):
        if _conv.shortcut_native_ok(x, conv):
            return _conv.shortcut_conv1x1(x, conv, link=x.grad_fn)
        return _LinkedConv.apply(x, conv.weight, conv.stride, conv.padding, conv.dilation, conv.groups, x.grad_fn)
    if torch.is_grad_enabled() and _conv.shortcut_native_ok(x, conv):
        return _conv.shortcut_conv1x1(x, conv)  # e.g. ResNet layer1's projection of the max-pool output
    return conv(x)


_DEFERRED = {"last": None}  # (data_ptr of the unwritten output, apply arguments) of the last deferred forward


def bn_act(x: torch.Tensor, bn: nn.modules.batchnorm._BatchNorm, residual: Optional[torch.Tensor] = None,
           relu: bool = True, shortcut_link: bool = False, defer_apply: bool = False,
           defer_affine: bool = False) -> torch.Tensor:
    """``act(bn(x) + residual)`` with the module's parameters/buffers and train/eval semantics.

    ``shortcut_link``: the caller guarantees ``residual`` is an identity shortcut, i.e. also the
    input of a differentiable op upstream of ``x`` (the block's first conv).  When ``residual`` was
    produced by this fused op, its gradient then travels to the producer's backward directly."""
    use_batch_stats = bn.training or not bn.track_running_stats
    rm = bn.running_mean if (bn.track_running_stats and bn.training) else None
    rv = bn.running_var if (bn.track_running_stats and bn.training) else None
    res_ok = residual is None or (residual.shape == x.shape and residual.device == x.device)
    _conv.materialize_fwd_apply(x)  # inputs whose producing BN apply was deferred but never staged
    # a residual whose BN apply was deferred (defer_affine) is computed inside this apply when the
    # fused training path runs; anything else materialises it
    aff = getattr(residual, "_det_affine_apply", None) if residual is not None else None
    res_affine = None
    if (aff is not None and not aff[3] and _nhwc_ok(x) and res_ok and use_batch_stats and relu and not shortcut_link
            and x.dtype == torch.bfloat16 and residual.dtype == x.dtype):
        residual._det_affine_apply = None
        res_affine = aff[:3]
    else:
        _conv.materialize_fwd_apply(residual)
    if _nhwc_ok(x) and res_ok:
        if use_batch_stats:
            nbt = bn.num_batches_tracked if (bn.training and bn.track_running_stats) else None
            link = None
            if (shortcut_link and SHORTCUT_LINK and residual is not None and torch.is_grad_enabled() and residual.requires_grad
                    and isinstance(residual.grad_fn, _BNActTrain._backward_cls) and residual.dtype == x.dtype
                    and residual.is_contiguous(memory_format=torch.channels_last if x.dim() == 4
                                               else torch.contiguous_format)):
                link = residual.grad_fn
                residual = residual.detach()
            defer = bool(defer_apply and _conv.DEFER_FWD_APPLY and torch.is_grad_enabled())
            daff = bool(defer_affine and _conv.DEFER_AFFINE_APPLY and torch.is_grad_enabled() and residual is None)
            out = _BNActTrain.apply(x, residual, bn.weight, bn.bias, rm, rv, nbt, bn.momentum, bn.eps, relu, link,
                                    defer, res_affine, daff)
            last, _DEFERRED["last"] = _DEFERRED["last"], None
            if last is not None:
                if last[0] != out.data_ptr():
                    raise RuntimeError("deferred BN apply: output buffer changed across autograd")
                if last[1][0] == "affine":
                    out._det_affine_apply = last[1][1:]
                else:
                    out._det_fwd_apply = last[1]
            return out
        needs_grad = torch.is_grad_enabled() and (
            x.requires_grad or (residual is not None and residual.requires_grad)
            or (bn.weight is not None and bn.weight.requires_grad))
        if not needs_grad:
            return _apply_frozen(x, bn, residual, relu)
    if x.device.type == "cuda":
        FALLBACKS["count"] += 1
    if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    momentum = bn.momentum
    if momentum is None and bn.training and bn.track_running_stats:
        momentum = 1.0 / float(bn.num_batches_tracked.item())
    return reference_bn_act(x, residual, bn.weight, bn.bias,
                            bn.running_mean if not use_batch_stats or bn.training else None,
                            bn.running_var if not use_batch_stats or bn.training else None,
                            use_batch_stats, momentum if momentum is not None else 0.1, bn.eps, relu)


def _apply_frozen(x, bn, residual, relu):
    M, C = _rows(x)
    rstd = torch.rsqrt(bn.running_var.float() + bn.eps)
    w = bn.weight.float() if bn.weight is not None else torch.ones_like(rstd)
    b = bn.bias.float() if bn.bias is not None else torch.zeros_like(rstd)
    scale = (w * rstd).contiguous()
    shift = (b - bn.running_mean.float() * scale).contiguous()
    fmt = torch.channels_last if x.dim() == 4 else torch.contiguous_format
    y = torch.empty_like(x, memory_format=fmt)
    if residual is not None:
        residual = residual.to(x.dtype).contiguous(memory_format=fmt)
    _lib.check(
        _lib.get_lib().det_bn_apply(_stream(x), _DT[x.dtype], x.data_ptr(), _ptr(residual), y.data_ptr(), M, C,
                                    scale.data_ptr(), shift.data_ptr(), int(bool(relu))),
        "bn_apply",
    )
    return y


class BatchNormAct2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` + optional residual add + optional ReLU in one fused HIP pass."""

    def __init__(self, num_features: int, relu: bool = True, fused: bool = True, **kw) -> None:
        super().__init__(num_features, **kw)
        self.relu = relu
        self.fused = fused  # False: stock torch/MIOpen BN + separate add/ReLU (A/B comparisons)

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,  # type: ignore[override]
                shortcut_link: bool = False, defer_apply: bool = False, defer_affine: bool = False) -> torch.Tensor:
        if self.fused:
            return bn_act(x, self, residual, self.relu, shortcut_link, defer_apply, defer_affine)
        _conv.materialize_fwd_apply(residual)
        y = super().forward(x)
        if residual is not None:
            y = y + residual
        return F.relu(y) if self.relu else y

    def extra_repr(self) -> str:
        return super().extra_repr() + f", relu={self.relu}"
