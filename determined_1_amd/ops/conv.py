"""Python entry points for the 1x1-convolution GEMMs of ``csrc/det_conv.hip``.

All tensors are row-major 2-D views of channels_last activations: ``x2d`` is ``[N*H*W, C]``.
The kernels need bf16, 16-byte aligned, contiguous operands with channel counts that are
multiples of 64 (every 1x1 conv of ResNet-50 qualifies); ``supported()`` says whether a call
can take the HIP path.  On CPU tensors the functions compute the same result with torch ops
(fp32 accumulate), which is what the unit tests compare against.
"""
import ctypes
import os
from typing import NamedTuple, Optional, Tuple

import torch

from determined_1_amd.ops import _lib
from determined_1_amd.ops.arena import side_work
from determined_1_amd.ops.functional import is_gpu

Gather = Tuple[int, int, int, int]  # (Ho, Wo, Hi, Wi) of a 1x1 stride-2 conv


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _wgrad_target(weight: torch.Tensor, needed: bool, gpu: bool, dy_numel: int,
                  memory_format: torch.memory_format = torch.contiguous_format) -> Tuple[Optional[torch.Tensor], bool]:
    """(dw, side) for a conv weight gradient: the parameter's arena slot when its GradSink offers
    one (arena.landing_buffer), else a fresh tensor; ``side`` = the gradient may be computed on the
    side stream (arena.side_work: only into the arena slot, whose readers all join first)."""
    if not needed:
        return None, False
    from determined_1_amd.ops import arena

    buf = arena.landing_buffer(weight)
    if buf is not None and buf.is_contiguous(memory_format=memory_format) and \
            buf.dtype in (torch.bfloat16, torch.float32):
        return buf, arena.SIDE_WGRAD and gpu and buf.dtype == weight.dtype and dy_numel >= arena.SIDE_MIN_ELEMS
    dt = weight.dtype if weight.dtype in (torch.bfloat16, torch.float32) else torch.float32
    return torch.empty(weight.shape, dtype=dt, device=weight.device, memory_format=memory_format), False


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def supported(x2d: torch.Tensor, w2d: torch.Tensor) -> bool:
    return (x2d.dtype == torch.bfloat16 and w2d.dtype == torch.bfloat16 and x2d.dim() == 2 and w2d.dim() == 2
            and x2d.shape[1] % 64 == 0 and w2d.shape[0] % 64 == 0 and w2d.shape[1] == x2d.shape[1]
            and x2d.is_contiguous() and w2d.is_contiguous()
            and x2d.data_ptr() % 16 == 0 and w2d.data_ptr() % 16 == 0)


def rows_per_block(n: int) -> int:
    return int(_lib.get_lib().det_conv_nt_rows_per_block(int(n)))


def _gather_rows(x2d: torch.Tensor, gather: Optional[Gather], m: int) -> torch.Tensor:
    if gather is None:
        return x2d
    ho, wo, hi, wi = gather
    n = m // (ho * wo)
    x4 = x2d.view(n, hi, wi, -1)
    return x4[:, ::2, ::2, :].reshape(m, -1)


def _affine_relu_ref(x: torch.Tensor, scale: Optional[torch.Tensor], shift: Optional[torch.Tensor]) -> torch.Tensor:
    if scale is None:
        return x
    return torch.relu(x.float() * scale + shift).to(x.dtype)


def conv1x1_nt(a2d: torch.Tensor, b2d: torch.Tensor, m: Optional[int] = None, scale: Optional[torch.Tensor] = None,
               shift: Optional[torch.Tensor] = None, stats: bool = False, gather: Optional[Gather] = None,
               out: Optional[torch.Tensor] = None, res: Optional[torch.Tensor] = None, aout: Optional[torch.Tensor] = None,
               abits: Optional[torch.Tensor] = None, res_scale: Optional[torch.Tensor] = None,
               res_shift: Optional[torch.Tensor] = None
               ) -> Tuple[torch.Tensor, Optional[Tuple[torch.Tensor, torch.Tensor, int]]]:
    """``C = op(A) . B^T`` with ``op(A) = relu(A*scale+shift)`` when scale/shift are given.

    Returns ``(C [M, N] bf16, partials)`` where partials is ``(pmean, pm2, rows_per_block)`` of the
    bf16-rounded C when ``stats`` (the BatchNorm statistics of the conv output), else None."""
    n, k = b2d.shape
    if m is None:
        m = a2d.shape[0] if gather is None else None
    assert m is not None
    if not is_gpu(a2d):
        a = _affine_relu_ref(_gather_rows(a2d, gather, m), scale, shift)
        c = (a.float() @ b2d.float().t()).to(a2d.dtype)
        parts = None
        if stats:
            rpb = 128
            nrb = (m + rpb - 1) // rpb
            cf = c.float()
            pad = nrb * rpb - m
            blocks = torch.cat([cf, cf.new_zeros(pad, n)]).view(nrb, rpb, n)
            cnt = torch.full((nrb, 1), float(rpb))
            cnt[-1, 0] = float(m - (nrb - 1) * rpb)
            mean = blocks.sum(1) / cnt
            valid = (torch.arange(rpb).view(1, rpb, 1) < cnt.view(nrb, 1, 1))
            m2 = (((blocks - mean.unsqueeze(1)) ** 2) * valid).sum(1)
            parts = (mean.contiguous(), m2.contiguous(), rpb)
        if out is not None:
            out.copy_(c)
            c = out
        return c, parts
    c = out if out is not None else torch.empty(m, n, dtype=a2d.dtype, device=a2d.device)
    parts = None
    pm = pq = None
    if stats:
        rpb = rows_per_block(n)
        nrb = (m + rpb - 1) // rpb
        pm = torch.empty(nrb, n, dtype=torch.float32, device=a2d.device)
        pq = torch.empty(nrb, n, dtype=torch.float32, device=a2d.device)
        parts = (pm, pq, rpb)
    g = gather or (0, 0, 0, 0)
    _lib.check(_lib.get_lib().det_conv_nt(_stream(a2d), a2d.data_ptr(), b2d.data_ptr(), c.data_ptr(), int(m), int(n),
                                          int(k), _ptr(scale), _ptr(shift), _ptr(pm), _ptr(pq), *[int(v) for v in g],
                                          _ptr(res), _ptr(aout), _ptr(abits), _ptr(res_scale), _ptr(res_shift)),
               "conv_nt")
    return c, parts


def conv1x1_wgrad(dy2d: torch.Tensor, x2d: torch.Tensor, out: torch.Tensor, scale: Optional[torch.Tensor] = None,
                  shift: Optional[torch.Tensor] = None, gather: Optional[Gather] = None,
                  out_scale: float = 1.0) -> torch.Tensor:
    """``out[N, K] = out_scale * dY[M, N]^T . op(X)[M, K]`` (fp32 accumulation, split over M)."""
    m, n = dy2d.shape
    k = x2d.shape[1]
    if not is_gpu(dy2d):
        xg = _affine_relu_ref(_gather_rows(x2d, gather, m), scale, shift)
        res = (dy2d.float().t() @ xg.float()) * out_scale
        out.copy_(res.view_as(out))
        return out
    if WGRAD_RING and scale is None and gather is None and ring_wgrad_1x1(n, k) and \
            int(_lib.get_lib().det_igemm_wgrad_ws_elems(m, n, k, 0)) > 0:
        # a stride-1 1x1 conv is the R = S = 1 case of the ring wgrad over one [1, M] "image"
        return conv_wgrad(dy2d.view(1, 1, m, n).permute(0, 3, 1, 2), x2d.view(1, 1, m, k).permute(0, 3, 1, 2),
                          out.view(n, k), 1, 1, 1, 0, out_scale=out_scale)
    ws = torch.empty(int(_lib.get_lib().det_conv_tn_ws_elems(m, n, k)), dtype=torch.float32, device=dy2d.device)
    g = gather or (0, 0, 0, 0)
    code = 1 if out.dtype == torch.bfloat16 else 0
    assert out.dtype in (torch.bfloat16, torch.float32) and out.is_contiguous() and out.numel() == n * k
    _lib.check(_lib.get_lib().det_conv_tn(_stream(dy2d), dy2d.data_ptr(), x2d.data_ptr(), out.data_ptr(), code, int(m),
                                          int(n), int(k), _ptr(scale), _ptr(shift), ws.data_ptr(), float(out_scale),
                                          *[int(v) for v in g]),
               "conv_tn")
    return out


# ------------------------------------------------------------------------------------------------
# pipelined implicit-GEMM convolution (csrc/det_igemm.hip)
# ------------------------------------------------------------------------------------------------
_ZERO = {}


def _zero_page(dev: torch.device) -> torch.Tensor:
    """256 zero bytes on ``dev``: the source the conv gather reads for padding taps and row tails."""
    z = _ZERO.get(dev)
    if z is None:
        z = _ZERO[dev] = torch.zeros(128, dtype=torch.bfloat16, device=dev)
    return z


def krsc(w: torch.Tensor) -> torch.Tensor:
    """Conv weight [Cout, Cin, R, S] as the [Cout, R*S*Cin] KRSC matrix det_igemm reads (a view for
    channels_last weights)."""
    co = w.shape[0]
    return w.permute(0, 2, 3, 1).reshape(co, -1).contiguous()


def igemm_supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 64 == 0 and w.shape[0] % 64 == 0
            and x.is_contiguous(memory_format=torch.channels_last))


# 3x3 / stride-1 convolutions with at most this many output channels run on the halo-patch kernel
# (det_igemm.hip conv3p: the input staged once per 256-pixel tile instead of once per tap).  Off by
# default: measured slower than igemm3 at every ResNet-50 shape (64 ch @56: fwd 0.317 vs 0.292 ms,
# dgrad 0.279 vs 0.259; 128 ch @28: fwd 0.253 vs 0.184) and -1.5 % on the whole step
# (profiles/r4_conv3x3_microbench.jsonl, r4_conv3p_ab.jsonl).
CONV3P_MAX_N = int(os.environ.get("DET_CONV3P_MAX_N", "0"))
CONV3P_COUNTS = {"fwd": 0, "dgrad": 0, "wgrad": 0}


def conv3p_ok(cin: int, cout: int, r: int, s: int, stride: int, pad: int) -> bool:
    return (r == 3 and s == 3 and stride == 1 and pad == 1 and cin % 32 == 0 and cout % 64 == 0
            and cout <= CONV3P_MAX_N)


def conv3p(x: torch.Tensor, wk: torch.Tensor, cout: int, stats: bool = False, pro=None, bnb=None):
    """3x3 / stride-1 / pad-1 conv of channels_last bf16 ``x`` with the KRSC weight ``wk``
    [Cout, 9*Cin] on det_conv3p.  ``pro`` = (scale, shift): the input operand is relu(x*scale+shift)
    (a BatchNorm+ReLU applied while staging).  ``bnb`` = (bn_x, mean, scale, shift): the output is the
    input gradient feeding that BN's backward; returns (masked gradient, (psum, psumx, 256)).
    Otherwise returns (y, BN statistics partials of y or None).  Returns None when a tile's halo
    patch does not fit (very wide images)."""
    nb, cin, h, w = x.shape
    m = nb * h * w
    lib = _lib.get_lib()
    y = torch.empty((nb, cout, h, w), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    nrb = (m + 255) // 256
    pm = pq = None
    bn = [None] * 6
    if stats:
        pm = torch.empty(nrb, cout, dtype=torch.float32, device=x.device)
        pq = torch.empty(nrb, cout, dtype=torch.float32, device=x.device)
    if bnb is not None:
        bx, mean, sc, sh = bnb
        pm_b = torch.empty(nrb, cout, dtype=torch.float32, device=x.device)
        pq_b = torch.empty(nrb, cout, dtype=torch.float32, device=x.device)
        bn = [bx.data_ptr(), mean.data_ptr(), sc.data_ptr(), sh.data_ptr(), pm_b.data_ptr(), pq_b.data_ptr()]
    rc = lib.det_conv3p(_stream(x), x.data_ptr(), wk.data_ptr(), y.data_ptr(), int(nb), int(h), int(w), int(cin),
                        int(cout), _ptr(pro[0]) if pro else None, _ptr(pro[1]) if pro else None, _ptr(pm), _ptr(pq),
                        *bn, 0)
    if rc == -6:
        return None
    _lib.check(rc, "conv3p")
    if bnb is not None:
        CONV3P_COUNTS["dgrad"] += 1
        return y, (pm_b, pq_b, 256)
    CONV3P_COUNTS["fwd"] += 1
    return y, ((pm, pq, 256) if stats else None)


CONV3P_WGRAD = os.environ.get("DET_CONV3P_WGRAD", "1") != "0"  # A/B switch: MIOpen's wrw kernels
CONV3P_WGRAD_MAX_C = int(os.environ.get("DET_CONV3P_WGRAD_MAX_C", "64"))


def conv3p_wgrad_ok(cin: int, cout: int, r: int, s: int, stride: int, pad: int) -> bool:
    # 64 channels only: 0.272 ms vs MIOpen 0.334 at 56x56; at 128 the ring (0.224) is ahead (0.255)
    return (CONV3P_WGRAD and r == 3 and s == 3 and stride == 1 and pad == 1 and cin % 64 == 0 and cout % 64 == 0
            and cin <= CONV3P_WGRAD_MAX_C)


def conv3p_wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor, out_scale: float = 1.0) -> bool:
    """Weight gradient of a 3x3 / stride-1 / pad-1 conv into ``out`` (contiguous [Cout, 9*Cin] KRSC
    view, bf16 or fp32) on det_conv3p_wgrad (the halo patch staged once for all 9 taps).  False when
    a chunk's patch does not fit (the caller falls back)."""
    nb, cin, h, w = x.shape
    cout = dy.shape[1]
    m = nb * h * w
    lib = _lib.get_lib()
    ws = torch.empty(int(lib.det_conv3p_wgrad_ws_elems(m, cout, cin)), dtype=torch.float32, device=dy.device)
    rc = lib.det_conv3p_wgrad(_stream(dy), dy.data_ptr(), x.data_ptr(), out.data_ptr(),
                              1 if out.dtype == torch.bfloat16 else 0, int(nb), int(h), int(w), int(cin), int(cout),
                              ws.data_ptr(), float(out_scale))
    if rc == -6:
        return False
    _lib.check(rc, "conv3p_wgrad")
    CONV3P_COUNTS["wgrad"] += 1
    return True


def igemm_conv(x: torch.Tensor, w: torch.Tensor, stride: int = 1, pad: int = 0, stats: bool = False,
               w_krsc: Optional[torch.Tensor] = None, cfg: int = 0) -> Tuple[torch.Tensor, Optional[Tuple[torch.Tensor, torch.Tensor, int]]]:
    """``conv2d(x, w, stride, pad)`` for channels_last bf16 ``x`` (Cin % 32 == 0) and Cout % 64 == 0.
    Returns (y channels_last bf16, BN statistics partials of y when ``stats``).  ``w_krsc``: the
    weight already in [Cout, R*S*Cin] form (e.g. the flipped/transposed dgrad weight).  ``cfg``:
    det_igemm tile configuration (0 = the measured per-shape choice)."""
    nb, cin, hi, wi = x.shape
    cout, _, r, s = w.shape
    ho = (hi + 2 * pad - r) // stride + 1
    wo = (wi + 2 * pad - s) // stride + 1
    m = nb * ho * wo
    if not is_gpu(x):
        y = torch.nn.functional.conv2d(x.float(), w.float(), stride=stride, padding=pad).to(x.dtype)
        y = y.contiguous(memory_format=torch.channels_last)
        parts = None
        if stats:
            y2 = y.permute(0, 2, 3, 1).reshape(m, cout)
            _, parts = conv1x1_nt(y2, torch.eye(cout, dtype=y.dtype), stats=True)  # exact copy + stats
        return y, parts
    wk = krsc(w) if w_krsc is None else w_krsc
    assert wk.dtype == torch.bfloat16 and wk.is_contiguous() and wk.shape == (cout, r * s * cin)
    if cfg == 0 and conv3p_ok(cin, cout, r, s, stride, pad) and x.data_ptr() % 16 == 0:
        res = conv3p(x, wk, cout, stats=stats)
        if res is not None:
            return res
    y = torch.empty((nb, cout, ho, wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    parts = None
    pm = pq = None
    if stats:
        rpb = int(_lib.get_lib().det_igemm_rows_per_block_cfg(int(cout), int(cfg)))
        nrb = (m + rpb - 1) // rpb
        pm = torch.empty(nrb, cout, dtype=torch.float32, device=x.device)
        pq = torch.empty(nrb, cout, dtype=torch.float32, device=x.device)
        parts = (pm, pq, rpb)
    _lib.check(_lib.get_lib().det_igemm_conv_cfg(_stream(x), x.data_ptr(), wk.data_ptr(), y.data_ptr(),
                                                 _zero_page(x.device).data_ptr(), int(m), int(cout), int(cin), int(hi),
                                                 int(wi), int(ho), int(wo), int(r), int(s), int(stride), int(pad),
                                                 _ptr(pm), _ptr(pq), int(cfg)),
               "igemm_conv")
    return y, parts


def _dw_ok(w: torch.Tensor) -> bool:
    return is_gpu(w) and w.dtype in (torch.float32, torch.bfloat16) and w.is_contiguous(memory_format=torch.channels_last)


# Batched flips (det_conv_dgrad_weight_multi): every R x S conv forward that will need its input
# gradient registers its weight (_DW_PENDING); the first dgrad_weight call of the backward flips all
# pending weights in one launch into _DW_READY, and each later call takes its own.  Entries are keyed
# by (data_ptr, shape, dtype) and computed during the backward from the weights as they are then --
# a weight changes only between backward passes (optimizer), and its next forward drops its old
# entry -- so no flip is ever older than the forward that uses it.  DW_BATCH = False: one launch each.
DW_BATCH = os.environ.get("DET_DW_BATCH", "1") != "0"
_DW_PENDING: dict = {}
_DW_READY: dict = {}
DW_COUNTS = {"batched_launches": 0, "served": 0}


def _dw_key(w: torch.Tensor):
    return (w.data_ptr(), tuple(w.shape), w.dtype)


def dgrad_weight_register(w: torch.Tensor) -> None:
    """Called by the forward of an R x S conv whose backward will flip ``w`` (see DW_BATCH)."""
    if DW_BATCH and _dw_ok(w):
        key = _dw_key(w)
        _DW_READY.pop(key, None)
        _DW_PENDING[key] = w


def _dgrad_weight_flush(w: torch.Tensor) -> None:
    _DW_PENDING[_dw_key(w)] = w
    items = list(_DW_PENDING.items())
    _DW_PENDING.clear()
    ws, outs, dims = [], [], []
    for key, t in items:
        k, c, r, s = t.shape
        out = torch.empty(c, r * s * k, dtype=torch.bfloat16, device=t.device)
        _DW_READY[key] = out
        ws.append(t.data_ptr())
        outs.append(out.data_ptr())
        dims += [k, c, r, s, 1 if t.dtype == torch.bfloat16 else 0]
    wa = (ctypes.c_int64 * len(ws))(*ws)
    oa = (ctypes.c_int64 * len(outs))(*outs)
    da = (ctypes.c_int * len(dims))(*dims)
    _lib.check(_lib.get_lib().det_conv_dgrad_weight_multi(_stream(w), len(ws), wa, oa, da), "conv_dgrad_weight_multi")
    DW_COUNTS["batched_launches"] += 1


def dgrad_weight(w: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, R, S] -> the [Cin, R*S*Cout] KRSC weight whose forward conv (stride 1, pad
    (R-1)/2) of dY is the input gradient: W'[c][r][s][k] = W[k][c][R-1-r][S-1-s].  One HIP
    transpose launch for channels_last fp32/bf16 weights on the GPU, or one for all the weights
    registered by their forwards (DW_BATCH)."""
    k, c, r, s = w.shape
    if DW_BATCH and _dw_ok(w) and (_DW_PENDING or _DW_READY):
        key = _dw_key(w)
        if key not in _DW_READY:
            _dgrad_weight_flush(w)
        DW_COUNTS["served"] += 1
        return _DW_READY.pop(key)
    if _dw_ok(w):
        out = torch.empty(c, r * s * k, dtype=torch.bfloat16, device=w.device)
        _lib.check(_lib.get_lib().det_conv_dgrad_weight(_stream(w), w.data_ptr(), 1 if w.dtype == torch.bfloat16 else 0,
                                                         out.data_ptr(), int(k), int(c), int(r), int(s)),
                   "conv_dgrad_weight")
        return out
    return w.flip(2, 3).permute(1, 2, 3, 0).reshape(c, -1).to(torch.bfloat16).contiguous()


WGRAD_RING = True  # det_igemm_wgrad (LDS-DMA ring, transposed reads) vs det_conv's register-staged gemm_tn
WGRAD_COUNTS = {"ring": 0, "slab": 0}
# 1x1 weight-gradient shapes (Cout, Cin) where the ring clearly beats gemm_tn at ResNet-50 / batch 512
# (0.105 vs 0.198 ms at 64x64 / 56x56, 0.088 vs 0.20 ms at 2048x512 / 7x7,
# profiles/r3_wgrad_ring_sweep.jsonl); the others stay on gemm_tn (within +-5 %, and the in-step A/B
# of routing them all to the ring lost 1.4 ms, profiles/r3_resnet50_ring_wgrad_all_steady.csv).
_RING_WGRAD_1X1 = {(64, 64), (2048, 512), (512, 2048)}
RING_WGRAD_1X1_ALL = False


def ring_wgrad_1x1(cout: int, cin: int) -> bool:
    return WGRAD_RING and (RING_WGRAD_1X1_ALL or (cout, cin) in _RING_WGRAD_1X1)


def conv_wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor, r: int, s: int, stride: int, pad: int,
               out_scale: float = 1.0, cfg: int = 0) -> torch.Tensor:
    """Weight gradient of a conv: ``out`` (contiguous [Cout, R*S*Cin] KRSC view, bf16 or fp32) =
    out_scale * dY^T . im2col(X) as split-pixel fp32 slabs reduced by a second launch: on
    det_igemm_wgrad (``WGRAD_RING``; ``cfg`` its tile configuration, 0 = automatic, -1 = force the
    older det_conv gemm_tn path) when a tile fits the shape, else on det_conv's gemm_tn."""
    nb, cin, hi, wi = x.shape
    cout, ho, wo = dy.shape[1], dy.shape[2], dy.shape[3]
    m = nb * ho * wo
    if not is_gpu(dy):
        g = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, r, s), dy.float(), stride=stride, padding=pad)
        out.copy_((g * out_scale).permute(0, 2, 3, 1).reshape(out.shape))
        return out
    assert out.dtype in (torch.bfloat16, torch.float32) and out.is_contiguous() and out.numel() == cout * r * s * cin
    lib = _lib.get_lib()
    if WGRAD_RING and cfg >= 0:
        n_ws = int(lib.det_igemm_wgrad_ws_elems(m, cout, r * s * cin, int(cfg)))
        if n_ws > 0 and dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0:
            ws = torch.empty(n_ws, dtype=torch.float32, device=dy.device)
            _lib.check(lib.det_igemm_wgrad(_stream(dy), dy.data_ptr(), x.data_ptr(), out.data_ptr(),
                                           1 if out.dtype == torch.bfloat16 else 0, int(m), int(cout), int(cin), int(hi),
                                           int(wi), int(ho), int(wo), int(r), int(s), int(stride), int(pad), ws.data_ptr(),
                                           float(out_scale), int(cfg)),
                       "igemm_wgrad")
            WGRAD_COUNTS["ring"] += 1
            return out
        if cfg > 0:
            _lib.check(-6, "igemm_wgrad (cfg %d does not tile [%d, %d])" % (cfg, cout, r * s * cin))
    WGRAD_COUNTS["slab"] += 1
    ws = torch.empty(int(lib.det_conv_tn_ws_elems(m, cout, r * s * cin)), dtype=torch.float32, device=dy.device)
    _lib.check(lib.det_conv_wgrad(_stream(dy), dy.data_ptr(), x.data_ptr(), out.data_ptr(),
                                  1 if out.dtype == torch.bfloat16 else 0, int(m), int(cout), int(cin), int(hi), int(wi),
                                  int(ho), int(wo), int(r), int(s), int(stride), int(pad), ws.data_ptr(),
                                  float(out_scale)),
               "conv_wgrad")
    return out


# ------------------------------------------------------------------------------------------------
# autograd: stride-1 1x1 convolution on channels_last bf16 activations
# ------------------------------------------------------------------------------------------------
COUNTS = {"native": 0, "fallback": 0}
ENABLED = True  # A/B switch (models.resnet.NATIVE_CONV1X1 toggles it)
DGRAD_BT = True  # 1x1 input gradients read the weight untransposed (no per-call transpose copy)
# 1x1 forward shapes (Cin, Cout) -> det_igemm tile configuration where the LDS-DMA implicit GEMM
# beat the register-staged gemm_nt by >= 7 % at ResNet-50 / batch 512 (profiles/r3_igemm_cfgs_1x1.jsonl:
# 0.063 vs 0.084 ms at 2048->512, 0.123 vs 0.136 at 256->1024, ...); the rest stay on gemm_nt.
IGEMM_FWD_1X1 = {(256, 1024): 8, (2048, 512): 8, (1024, 512): 8, (512, 256): 8, (1024, 256): 8}
if os.environ.get("DET_NT_WIDE") == "1":  # A/B: the layer-3 expansion on det_conv's occupancy-3 wide tiles
    IGEMM_FWD_1X1.pop((256, 1024))


def _attach_partials(y: torch.Tensor, parts: Optional[Tuple[torch.Tensor, torch.Tensor, int]]) -> None:
    """Hand the BN statistics partials of ``y`` to the BatchNorm that consumes it (ops/norm.py)."""
    if parts is not None:
        y._det_bn_parts = (y.data_ptr(), parts)  # type: ignore[attr-defined]


def take_partials(x: torch.Tensor) -> Optional[Tuple[torch.Tensor, torch.Tensor, int]]:
    p = getattr(x, "_det_bn_parts", None)
    if p is None or p[0] != x.data_ptr():
        return None
    return p[1]


# BatchNorm-backward fusion into the input-gradient GEMM of a 1x1 conv whose input is the output of
# a fused training BatchNorm(+add)(+ReLU) that has no other autograd consumer (ResNet bottleneck
# bn2 -> conv3; block output -> next block's conv1, whose identity / projection shortcut gradient
# arrives through the BN link).  The dgrad epilogue applies the ReLU mask (and adds the shortcut
# gradient), writes that masked gradient d and the BN's backward partial sums, so the BN backward
# is finalize + an unmasked apply and d doubles as the shortcut's gradient (det_conv_nt_bnbwd,
# det_bn_bwd_from_partials).  False: the separate partial pass (A/B).
FUSE_BN_BWD = True
FUSE_BN_BWD_MODES = (1, 2)  # 1: ReLU mask from x (bn2 -> conv3); 2: forward mask bits + shortcut gradient
BN_BWD_COUNTS = {"fused": 0, "unfused": 0}


def _bn_producer(x: torch.Tensor):
    """The fused-BN autograd node that produced ``x`` (None if not such an output)."""
    from determined_1_amd.ops.norm import _BNActTrain

    gf = x.grad_fn
    return gf if isinstance(gf, _BNActTrain._backward_cls) else None


def dgrad_1x1(dy2d: torch.Tensor, w2d: torch.Tensor, abn=None) -> torch.Tensor:
    """dX[M, Cin] = dY[M, Cout] . W[Cout, Cin] for a 1x1 conv.  On the GPU with ``DGRAD_BT`` the GEMM
    reads the weight as stored (transposed LDS reads), else through a transposed copy.  ``abn`` =
    (d, x, coef, out): dY is the deferred BN-backward apply of the consuming BN (see
    ``take_pending_apply``), staged by the GEMM and written to ``out`` (the 2-D view of dY)."""
    if DGRAD_BT and is_gpu(dy2d) and w2d.dtype == torch.bfloat16 and w2d.is_contiguous():
        m, k = dy2d.shape
        n = w2d.shape[1]
        dx = torch.empty(m, n, dtype=torch.bfloat16, device=dy2d.device)
        a_src, ax, acoef, aout = (dy2d, None, None, None) if abn is None else abn
        _lib.check(_lib.get_lib().det_conv_dgrad(_stream(dy2d), a_src.data_ptr(), w2d.data_ptr(), dx.data_ptr(), int(m),
                                                 int(n), int(k), _ptr(ax), _ptr(acoef), _ptr(aout)), "conv_dgrad")
        return dx
    assert abn is None
    return conv1x1_nt(dy2d, w2d.t().contiguous())[0]


# Deferred BatchNorm-backward apply (``DEFER_BN_APPLY``): a fused training BN whose input is the
# output of a native 1x1 conv (ResNet bn3 <- conv3) runs only its finalize and hands (d, x, coef) to
# that conv's backward, whose input-gradient GEMM computes dY = A d + B x + C while staging its A
# operand and writes it for the weight gradient: the apply pass and the GEMM's read of dY become one.
DEFER_BN_APPLY = os.environ.get("DET_DEFER_BN_APPLY", "1") != "0"
BN_APPLY_COUNTS = {"deferred": 0, "in_gemm": 0, "materialized": 0}


def take_pending_apply(ctx, dy: torch.Tensor):
    """(d, x, coef) of a BN backward deferred onto this conv node, checked against the gradient
    buffer ``dy`` it returned (None if nothing is pending)."""
    pend = getattr(ctx, "pending_bn_apply", None)
    ctx.pending_bn_apply = None
    if pend is None:
        return None
    buf, d, x, coef = pend
    if buf.data_ptr() != dy.data_ptr() or dy.shape != buf.shape:
        raise RuntimeError("deferred BN-backward apply: the gradient reached the conv in a different buffer")
    return d, x, coef


def materialize_pending_apply(dy: torch.Tensor, pend) -> None:
    d, x, coef = pend
    m = d.numel() // d.shape[1]
    _lib.check(_lib.get_lib().det_bn_bwd_apply_coef(_stream(d), 1 if d.dtype == torch.bfloat16 else 0, d.data_ptr(),
                                                    x.data_ptr(), int(m), int(d.shape[1]), coef.data_ptr(),
                                                    dy.data_ptr()), "bn_bwd_apply_coef")
    BN_APPLY_COUNTS["materialized"] += 1


# Deferred BatchNorm forward apply (``DEFER_FWD_APPLY``): a fused training BN(+residual)+ReLU whose
# output's first consumer is a native 1x1 conv (ResNet bn3 -> the next identity block's conv1;
# ``models.resnet`` marks those blocks) runs only its finalize and returns its output buffer
# unwritten, tagged ``_det_fwd_apply = (x, residual, scale, shift, mbits)``; the conv's forward GEMM
# computes relu(x*scale + shift + residual) while staging its A operand and writes it and its mask
# bits into the tagged buffers (det_conv.hip AFWD).  Any other first consumer materialises it.
DEFER_FWD_APPLY = os.environ.get("DET_DEFER_FWD_APPLY", "1") != "0"
FWD_APPLY_COUNTS = {"deferred": 0, "in_gemm": 0, "materialized": 0}


def materialize_fwd_apply(t: Optional[torch.Tensor]) -> None:
    """Write a deferred BN forward apply into ``t`` (no-op for untagged tensors)."""
    if t is None:
        return
    aff = getattr(t, "_det_affine_apply", None)
    if aff is not None:
        t._det_affine_apply = None
        materialize_affine_apply(t, aff)
    pend = getattr(t, "_det_fwd_apply", None)
    if pend is None:
        return
    t._det_fwd_apply = None
    x, res, scale, shift, mbits, rs, rh = pend
    m = x.numel() // x.shape[1]
    _lib.check(_lib.get_lib().det_bn_apply_res_mbits(_stream(x), x.data_ptr(), res.data_ptr(), t.data_ptr(), int(m),
                                                     int(x.shape[1]), scale.data_ptr(), shift.data_ptr(),
                                                     mbits.data_ptr(), _ptr(rs), _ptr(rh)), "bn_apply_res_mbits")
    FWD_APPLY_COUNTS["materialized"] += 1


# Deferred affine BN apply (``DEFER_AFFINE_APPLY``): a training BN without residual whose only
# consumer applies it itself runs only its finalize and returns its output unwritten, tagged
# ``_det_affine_apply = (x, scale, shift, relu)``.  Consumers: a residual BN(+ReLU) apply for ResNet's
# projection-shortcut BN (no ReLU, read only by bn3), which computes relu(bn3 + x * scale + shift)
# from x (det_norm.hip bn_apply_fwd RES 2, or det_conv.hip AFWD when bn3's apply is itself deferred
# onto the next conv); the stem max-pool for the stem BN + ReLU (det_pool.hip maxpool_fwd BNP).  The
# BN's apply pass (read x, write y) and the consumer's read of y become one read of x.
DEFER_AFFINE_APPLY = os.environ.get("DET_DEFER_AFFINE_APPLY", "1") != "0"
AFFINE_APPLY_COUNTS = {"deferred": 0, "in_residual": 0, "materialized": 0}


def materialize_affine_apply(t: torch.Tensor, aff) -> None:
    """Write ``t = [relu](x * scale + shift)`` (a deferred BN apply without residual, see
    ``DEFER_AFFINE_APPLY``)."""
    x, scale, shift = aff[:3]
    relu = len(aff) > 3 and bool(aff[3])
    m = x.numel() // x.shape[1]
    _lib.check(_lib.get_lib().det_bn_apply(_stream(x), 1 if x.dtype == torch.bfloat16 else 0, x.data_ptr(), None,
                                           t.data_ptr(), int(m), int(x.shape[1]), scale.data_ptr(), shift.data_ptr(),
                                           int(relu)), "bn_apply")
    AFFINE_APPLY_COUNTS["materialized"] += 1


class StridedGrad(NamedTuple):
    """Input gradient of a 1x1 stride-2 conv kept on its stride-2 grid: ``t`` [N, C, Ho, Wo]
    (channels_last) holds the values at the even (h, w) positions of the [N, C, Hi, Wi] input,
    zero elsewhere.  A producer's fused BN-backward epilogue reads it in place (det_conv.hip
    BnBwdEpi add_*); anything else materialises it (``full_res_grad``)."""
    t: torch.Tensor
    g: Gather  # (Ho, Wo, Hi, Wi)


def full_res_grad(extra, like: Optional[torch.Tensor] = None):
    """A shortcut gradient at the resolution of its input (``StridedGrad`` scattered into zeros)."""
    if not isinstance(extra, StridedGrad):
        return extra
    ho, wo, hi, wi = extra.g
    nb, c = extra.t.shape[0], extra.t.shape[1]
    full = torch.zeros((nb, hi, wi, c), dtype=extra.t.dtype, device=extra.t.device).permute(0, 3, 1, 2)
    full[:, :, ::2, ::2] = extra.t
    return full


def _fused_bn_dgrad(prod, dy2d: torch.Tensor, w2d: torch.Tensor, m: int, c: int, abn=None) -> Optional[torch.Tensor]:
    """dgrad with the producer BN's backward partials in the epilogue, or None when the producer
    cannot take it (no ReLU, the shortcut gradient not in yet, already fused, layout/dtype)."""
    mode = getattr(prod, "mask_mode", 0)
    if mode not in FUSE_BN_BWD_MODES or getattr(prod, "fused_bwd", None) is not None:
        return None
    expects = getattr(prod, "expects_extra", False)  # a linked shortcut also consumes the output
    if expects and getattr(prod, "extra_dy", None) is None:
        return None  # the identity/projection shortcut gradient has not been linked yet
    try:
        xb, mbits, _, stats = prod.saved_tensors
    except RuntimeError:
        return None
    if xb.dtype != torch.bfloat16 or xb.numel() != m * c or not xb.is_contiguous(memory_format=torch.channels_last):
        return None
    add = prod.extra_dy if expects else None
    sub = (0, 0, 0, 0)
    if isinstance(add, StridedGrad):  # a stride-2 projection shortcut's gradient, read on its grid
        sub, add = add.g, add.t
    if add is not None and (add.dtype != torch.bfloat16 or not add.is_contiguous(memory_format=torch.channels_last)):
        return None
    rpb = rows_per_block(c)
    nrb = (m + rpb - 1) // rpb
    psum = torch.empty(nrb, c, dtype=torch.float32, device=dy2d.device)
    psumx = torch.empty(nrb, c, dtype=torch.float32, device=dy2d.device)
    d = torch.empty(m, c, dtype=torch.bfloat16, device=dy2d.device)
    if abn is not None and not DGRAD_BT:
        return None
    wb = w2d if DGRAD_BT else w2d.t().contiguous()  # [Cout, Cin] as stored, or the transposed copy
    a_src, ax, acoef, aout = (dy2d, None, None, None) if abn is None else abn
    _lib.check(_lib.get_lib().det_conv_nt_bnbwd(
        _stream(dy2d), a_src.data_ptr(), wb.data_ptr(), d.data_ptr(), int(m), int(c), int(w2d.shape[0]), xb.data_ptr(),
        stats[0].data_ptr(), stats[2].data_ptr(), stats[3].data_ptr(), _ptr(mbits), _ptr(add), psum.data_ptr(),
        psumx.data_ptr(), int(mode), 1 if DGRAD_BT else 0, _ptr(ax), _ptr(acoef), _ptr(aout), *[int(v) for v in sub]),
        "conv_nt_bnbwd")
    prod.fused_bwd = (psum, psumx, rpb)
    if expects:
        prod.extra_dy = None  # consumed: summed into d
    return d


def _fused_bn_dgrad_rs(prod, dyc: torch.Tensor, wt: torch.Tensor, wd: torch.Tensor, pad: int) -> Optional[torch.Tensor]:
    """Stride-1 R x S input gradient on det_igemm with the producer BN's backward partials in its
    epilogue (mask mode 1: ReLU recomputed from the BN input; ResNet bn1 -> conv2), or None when the
    producer cannot take it."""
    if getattr(prod, "mask_mode", 0) != 1 or getattr(prod, "fused_bwd", None) is not None:
        return None
    try:
        xb, _, _, stats = prod.saved_tensors
    except RuntimeError:
        return None
    nb, cout, h, w_ = dyc.shape
    cin = wt.shape[0]
    m = nb * h * w_
    if xb.dtype != torch.bfloat16 or xb.shape != (nb, cin, h, w_) or not xb.is_contiguous(memory_format=torch.channels_last):
        return None
    r, s = wt.shape[2], wt.shape[3]
    if conv3p_ok(cout, cin, r, s, 1, pad):
        res = conv3p(dyc, wd, cin, bnb=(xb, stats[0], stats[2], stats[3]))
        if res is not None:
            d, fb = res
            prod.fused_bwd = fb
            return d
    lib = _lib.get_lib()
    cfg = 0
    rpb = int(lib.det_igemm_rows_per_block_cfg(int(cin), cfg))
    nrb = (m + rpb - 1) // rpb
    psum = torch.empty(nrb, cin, dtype=torch.float32, device=dyc.device)
    psumx = torch.empty(nrb, cin, dtype=torch.float32, device=dyc.device)
    d = torch.empty((nb, cin, h, w_), dtype=torch.bfloat16, device=dyc.device, memory_format=torch.channels_last)
    _lib.check(lib.det_igemm_conv_bnbwd(_stream(dyc), dyc.data_ptr(), wd.data_ptr(), d.data_ptr(),
                                        _zero_page(dyc.device).data_ptr(), int(m), int(cin), int(cout), int(h), int(w_),
                                        int(h), int(w_), int(r), int(s), 1, int(pad), xb.data_ptr(), stats[0].data_ptr(),
                                        stats[2].data_ptr(), stats[3].data_ptr(), psum.data_ptr(), psumx.data_ptr(),
                                        cfg), "igemm_conv_bnbwd")
    prod.fused_bwd = (psum, psumx, rpb)
    return d


DGRAD_S2_NATIVE = os.environ.get("DET_DGRAD_S2_NATIVE", "1") != "0"  # A/B switch: MIOpen's transposed conv


def dgrad_s2_ok(x: torch.Tensor, weight: torch.Tensor, stride: int, pad: int) -> bool:
    """The stride-2 3x3/pad-1 input gradient can run on det_igemm_dgrad_s2 (parity classes)."""
    cout, cin, r, s = weight.shape
    return (DGRAD_S2_NATIVE and stride == 2 and pad == 1 and r == 3 and s == 3 and cin % 64 == 0 and cout % 32 == 0
            and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0)


def igemm_dgrad_s2(dyc: torch.Tensor, weight: torch.Tensor, hi: int, wi: int, prod=None) -> torch.Tensor:
    """Input gradient [N, Cin, Hi, Wi] (channels_last bf16) of a 3x3 / stride-2 / pad-1 conv from dY
    (channels_last bf16): det_igemm_dgrad_s2, four parity-class implicit GEMMs over dY against taps of
    the flipped weight.  ``prod``: the fused BN(+ReLU) that produced the conv input (mask mode 1):
    its backward partials come from the GEMM epilogue (``prod.fused_bwd``) and the ReLU mask is
    applied to the returned gradient."""
    nb, cout, ho, wo = dyc.shape
    cin = weight.shape[1]
    if not is_gpu(dyc):  # CPU reference of the same computation
        g = torch.nn.grad.conv2d_input((nb, cin, hi, wi), weight.float(), dyc.float(), stride=2, padding=1)
        return g.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    lib = _lib.get_lib()
    wd = dgrad_weight(weight)  # [Cin, 9 * Cout]
    dx = torch.empty((nb, cin, hi, wi), dtype=torch.bfloat16, device=dyc.device, memory_format=torch.channels_last)
    bn = [None] * 6
    if prod is not None:
        xb, _, _, stats = prod.saved_tensors
        rpb = int(lib.det_igemm_dgrad_s2_rows_per_block(int(cin), 0))
        nrb = 4 * ((nb * ho * wo + rpb - 1) // rpb)
        psum = torch.empty(nrb, cin, dtype=torch.float32, device=dyc.device)
        psumx = torch.empty(nrb, cin, dtype=torch.float32, device=dyc.device)
        bn = [xb.data_ptr(), stats[0].data_ptr(), stats[2].data_ptr(), stats[3].data_ptr(), psum.data_ptr(),
              psumx.data_ptr()]
    _lib.check(lib.det_igemm_dgrad_s2(_stream(dyc), dyc.data_ptr(), wd.data_ptr(), dx.data_ptr(),
                                      _zero_page(dyc.device).data_ptr(), int(nb), int(ho), int(wo), int(cout), int(cin),
                                      *bn, 0), "igemm_dgrad_s2")
    if prod is not None:
        prod.fused_bwd = (psum, psumx, rpb)  # the BN backward sums the partials (any row order)
    return dx


def _bn_producer_s2_ok(prod, x: torch.Tensor) -> bool:
    if prod is None or getattr(prod, "mask_mode", 0) != 1 or getattr(prod, "fused_bwd", None) is not None:
        return False
    try:
        xb = prod.saved_tensors[0]
    except RuntimeError:
        return False
    return xb.dtype == torch.bfloat16 and xb.shape == x.shape and xb.is_contiguous(memory_format=torch.channels_last)


class _Conv1x1(torch.autograd.Function):
    """``conv2d(x, w)`` for a 1x1 stride-1 kernel as det_conv GEMMs: forward with the output's
    BatchNorm statistics in the epilogue, dgrad through the transposed weight (with the input's
    BatchNorm-backward partials in its epilogue when ``bn_producer`` is given), split-M wgrad that
    writes the weight gradient straight into its arena slot when the parameter has one."""

    @staticmethod
    def forward(ctx, x, weight, stats, bn_producer=None, fwd_apply=None):
        n, c, h, w_ = x.shape
        cout = weight.shape[0]
        x2 = x.permute(0, 2, 3, 1).reshape(-1, c)  # channels_last: a free view
        w2 = weight.reshape(cout, c)
        wb = w2 if w2.dtype == torch.bfloat16 else w2.to(torch.bfloat16)
        cfg = IGEMM_FWD_1X1.get((c, cout)) if is_gpu(x) else None
        if fwd_apply is not None:
            # x is the unwritten output of the producing BN: stage relu(bx*scale + shift + res) as
            # the A operand and write it (and its mask bits) into x (DEFER_FWD_APPLY)
            bx, res, scale, shift, mbits, rs, rh = fwd_apply
            y2, parts = conv1x1_nt(bx.permute(0, 2, 3, 1).reshape(-1, c), wb.contiguous(), scale=scale, shift=shift,
                                   stats=stats, res=res.permute(0, 2, 3, 1).reshape(-1, c), aout=x2, abits=mbits,
                                   res_scale=rs, res_shift=rh)
            y = y2.view(n, h, w_, cout).permute(0, 3, 1, 2)
            FWD_APPLY_COUNTS["in_gemm"] += 1
        elif cfg is not None and x.data_ptr() % 16 == 0:
            # LDS-DMA implicit GEMM (same BN-statistics epilogue, 256-row partial blocks)
            y, parts = igemm_conv(x, weight, stats=stats, w_krsc=wb.contiguous(), cfg=cfg)
        else:
            y2, parts = conv1x1_nt(x2, wb.contiguous(), stats=stats)
            y = y2.view(n, h, w_, cout).permute(0, 3, 1, 2)
        _attach_partials(y, parts)
        ctx.save_for_backward(x, weight)
        ctx.bn_producer = bn_producer
        # a consuming fused BN may defer its backward apply onto this node (take_pending_apply):
        # expansion convs only (ResNet conv3, Cout = 4 Cin), whose dgrad reads each staged A element
        # once; a reducing conv (conv1, Cout = Cin / 4) re-stages A per N tile and measured slower
        # than the separate apply (profiles/r3_bench_resnet50_defer_bn_apply_ab.jsonl)
        ctx.accepts_bn_apply = is_gpu(x) and DGRAD_BT and cout >= 2 * c
        ctx.pending_bn_apply = None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        n, c, h, w_ = x.shape
        cout = weight.shape[0]
        pend = take_pending_apply(ctx, dy)
        if pend is not None and not (ctx.needs_input_grad[0] and dy.dtype == torch.bfloat16
                                     and dy.is_contiguous(memory_format=torch.channels_last)):
            materialize_pending_apply(dy, pend)
            pend = None
        dy2 = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1).reshape(-1, cout)
        x2 = x.permute(0, 2, 3, 1).reshape(-1, c)
        dx = dw = None
        prod, ctx.bn_producer = ctx.bn_producer, None
        abn = None
        if pend is not None:  # dY = the deferred BN apply, computed in the dgrad's A staging into dy2
            d, bx, coef = pend
            abn = (d.permute(0, 2, 3, 1).reshape(-1, cout), bx, coef, dy2)
        dw, side = _wgrad_target(weight, ctx.needs_input_grad[1], is_gpu(dy2), dy2.numel())
        if side and pend is None:  # independent of the dgrad: fork before it
            with side_work(True, dy2, x2):
                conv1x1_wgrad(dy2, x2, dw.view(cout, c))
            side = None
        if ctx.needs_input_grad[0]:
            w2 = weight.reshape(cout, c).to(torch.bfloat16).contiguous()
            dx2 = _fused_bn_dgrad(prod, dy2, w2, n * h * w_, c, abn) if (prod is not None and is_gpu(dy2)) else None
            if dx2 is None:
                dx2 = dgrad_1x1(dy2, w2, abn)
                if prod is not None:
                    BN_BWD_COUNTS["unfused"] += 1
            else:
                BN_BWD_COUNTS["fused"] += 1
            if abn is not None:
                BN_APPLY_COUNTS["in_gemm"] += 1
            dx = dx2.view(n, h, w_, c).permute(0, 3, 1, 2)
        if dw is not None and side is not None:
            with side_work(side, dy2, x2):
                conv1x1_wgrad(dy2, x2, dw.view(cout, c))
            if dw.dtype != weight.dtype:
                dw = dw.to(weight.dtype)
        return dx, dw, None, None, None


class _BNReluConv1x1(torch.autograd.Function):
    """``conv1x1(relu(bn(x)))`` for a training-mode BatchNorm whose only consumer is a stride-1 1x1
    conv (ResNet bottleneck bn2 -> conv3).  The normalised activation is never materialised:

    forward : stats pass over ``x`` (det_bn_stats_train, no apply) -> GEMM whose A-operand prologue
              applies relu(x*scale+shift) while staging, with the output's BN statistics in its
              epilogue (for bn3).  Saves the apply pass (read x + write z) and the conv's read of z
              in exchange for reading x: 2 fewer activation passes per block.
    backward: dgrad GEMM -> dz; wgrad GEMM re-applies the same prologue to ``x`` (bit-identical z);
              det_bn_bwd with the ReLU mask recomputed from ``x`` (mask_mode 1) -> dx, dgamma, dbeta.
    """

    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, nbt, momentum, eps, weight):
        n, c, h, w_ = x.shape
        cout = weight.shape[0]
        m = n * h * w_
        lib = _lib.get_lib()
        x2 = x.permute(0, 2, 3, 1).reshape(m, c)
        stats = torch.empty((4, c), dtype=torch.float32, device=x.device)
        ws = torch.empty(int(lib.det_bn_ws_elems(m, c)), dtype=torch.float32, device=x.device)
        _lib.check(lib.det_bn_stats_train(
            _stream(x), 1, x.data_ptr(), m, c, _ptr(gamma), _ptr(beta), _ptr(running_mean), _ptr(running_var),
            _ptr(nbt), float(-1.0 if momentum is None else momentum), float(eps),
            stats[0].data_ptr(), stats[1].data_ptr(), stats[2].data_ptr(), stats[3].data_ptr(), ws.data_ptr()),
            "bn_stats_train")
        wb = weight.reshape(cout, c)
        wb = (wb if wb.dtype == torch.bfloat16 else wb.to(torch.bfloat16)).contiguous()
        y2, parts = conv1x1_nt(x2, wb, scale=stats[2], shift=stats[3], stats=True)
        y = y2.view(n, h, w_, cout).permute(0, 3, 1, 2)
        _attach_partials(y, parts)
        ctx.save_for_backward(x, gamma, stats, weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, stats, weight = ctx.saved_tensors
        n, c, h, w_ = x.shape
        cout = weight.shape[0]
        m = n * h * w_
        lib = _lib.get_lib()
        dy2 = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1).reshape(m, cout)
        x2 = x.permute(0, 2, 3, 1).reshape(m, c)
        dw = None
        if ctx.needs_input_grad[8]:
            from determined_1_amd.ops.arena import landing_buffer

            buf = landing_buffer(weight)
            if buf is not None and buf.is_contiguous() and buf.dtype in (torch.bfloat16, torch.float32):
                dw = buf
            else:
                dw = torch.empty(weight.shape, dtype=weight.dtype if weight.dtype in (torch.bfloat16, torch.float32)
                                 else torch.float32, device=weight.device)
            conv1x1_wgrad(dy2, x2, dw.view(cout, c), scale=stats[2], shift=stats[3])
            if dw.dtype != weight.dtype:
                dw = dw.to(weight.dtype)
        dz2 = dgrad_1x1(dy2, weight.reshape(cout, c).to(torch.bfloat16).contiguous())  # gradient of relu(bn(x))
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dgb = torch.empty((2, c), dtype=torch.float32, device=x.device) if gamma is not None else None
        ws = torch.empty(int(lib.det_bn_ws_elems(m, c)), dtype=torch.float32, device=x.device)
        _lib.check(lib.det_bn_bwd(
            _stream(x), 1, dz2.data_ptr(), None, x.data_ptr(), None, m, c, 1, _ptr(gamma),
            stats[0].data_ptr(), stats[1].data_ptr(), stats[2].data_ptr(), stats[3].data_ptr(), dx.data_ptr(), None,
            None if dgb is None else dgb[0].data_ptr(), None if dgb is None else dgb[1].data_ptr(), ws.data_ptr(), 1),
            "bn_bwd")
        dg = dgb[0] if dgb is not None and ctx.needs_input_grad[1] else None
        db = dgb[1] if dgb is not None and ctx.needs_input_grad[2] else None
        return dx, dg, db, None, None, None, None, None, dw


FUSED_COUNTS = {"bn_relu_conv1x1": 0, "fallback": 0, "stem": 0, "stem_fallback": 0, "stem_wgrad_patch": 0}


# ------------------------------------------------------------------------------------------------
# autograd: 3x3 (and other R x S) convolutions on the det_igemm implicit GEMM
# ------------------------------------------------------------------------------------------------
CONV3X3_COUNTS = {"native": 0, "fallback": 0, "dgrad_native": 0, "dgrad_miopen": 0, "wgrad_native": 0,
                  "wgrad_miopen": 0}
# R x S weight gradient: "auto" = det_igemm_wgrad (LDS-DMA ring) at Cin >= 256, where it beats MIOpen's
# wrw kernels (0.178 vs 0.202 ms at 256 ch / 14x14, and needs none of their zero-fill / cast launches),
# MIOpen's wrw below (0.33 vs 0.44 ms at 64 ch / 56x56; level at 128 ch in isolation, slower in the
# step; profiles/r3_wgrad_ring_sweep.jsonl); "native" forces the ring / gemm_tn path, "miopen" MIOpen.
WGRAD_RS_MODE = "auto"


class _ConvRS(torch.autograd.Function):
    """``conv2d(x, w, stride, pad)`` (R x S, no bias, groups 1) on channels_last bf16 activations:
    forward = det_igemm implicit GEMM with the output's BatchNorm statistics in its epilogue;
    input gradient = det_igemm forward conv of dY against the flipped/transposed weight (stride 1;
    strided convs keep MIOpen's transposed conv for the input gradient); weight gradient = det_conv
    split-M implicit GEMM with the im2col gather, written straight into the arena slot."""

    @staticmethod
    def forward(ctx, x, weight, stride, pad, stats, bn_producer=None):
        wk = krsc(weight.to(torch.bfloat16) if weight.dtype != torch.bfloat16 else weight)
        y, parts = igemm_conv(x, weight, stride=stride, pad=pad, stats=stats, w_krsc=wk)
        _attach_partials(y, parts)
        ctx.save_for_backward(x, weight)
        ctx.stride, ctx.pad = stride, pad
        ctx.bn_producer = bn_producer
        if ctx.needs_input_grad[0]:
            dgrad_weight_register(weight)  # flipped with the step's other R x S weights (DW_BATCH)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        stride, pad = ctx.stride, ctx.pad
        cout, cin, r, s = weight.shape
        dyc = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        # auto: the ring at >= 128 channels (at 128 a tie with MIOpen, 0.224 / 0.253 ms at stride 1 / 2,
        # profiles/r4_conv3x3_microbench.jsonl, and no library launch), the halo patch for the stride-1
        # 3x3 at 64 channels
        native_wgrad = WGRAD_RS_MODE == "native" or (WGRAD_RS_MODE == "auto" and WGRAD_RING and cin >= 128) or \
            (WGRAD_RS_MODE == "auto" and conv3p_wgrad_ok(cin, cout, r, s, stride, pad) and is_gpu(dyc))
        side = False
        if native_wgrad:
            dw, side = _wgrad_target(weight, ctx.needs_input_grad[1], is_gpu(dyc), dyc.numel(), torch.channels_last)
            if side:  # fork before the input gradient: the two only share dY
                with side_work(True, dyc, x):
                    _native_wgrad_rs(dyc, x, dw, stride, pad)
        if ctx.needs_input_grad[0]:
            if stride == 1 and 2 * pad == r - 1 and r == s:
                wd = dgrad_weight(weight)
                # (on the GPU only the shape of the second argument is read; the CPU reference
                # path convolves with it, so it gets the real flipped weight there)
                wt = weight.transpose(0, 1) if is_gpu(dyc) else weight.flip(2, 3).transpose(0, 1)
                prod, ctx.bn_producer = ctx.bn_producer, None
                dx = _fused_bn_dgrad_rs(prod, dyc, wt, wd, r - 1 - pad) if (prod is not None and is_gpu(dyc)) else None
                if dx is None:
                    dx, _ = igemm_conv(dyc, wt, stride=1, pad=r - 1 - pad, w_krsc=wd)
                    if prod is not None:
                        BN_BWD_COUNTS["unfused"] += 1
                else:
                    BN_BWD_COUNTS["fused"] += 1
                CONV3X3_COUNTS["dgrad_native"] += 1
            elif dgrad_s2_ok(x, weight, stride, pad) and is_gpu(dyc):
                prod, ctx.bn_producer = ctx.bn_producer, None
                fuse = _bn_producer_s2_ok(prod, x)
                dx = igemm_dgrad_s2(dyc, weight, x.shape[2], x.shape[3], prod if fuse else None)
                if prod is not None:
                    BN_BWD_COUNTS["fused" if fuse else "unfused"] += 1
                CONV3X3_COUNTS["dgrad_native"] += 1
            else:
                wb = weight.detach().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
                dx = torch.ops.aten.convolution_backward(dyc, x, wb, None, [stride, stride], [pad, pad], [1, 1], False,
                                                         [0, 0], 1, [True, False, False])[0]
                CONV3X3_COUNTS["dgrad_miopen"] += 1
        if ctx.needs_input_grad[1] and not native_wgrad:
            wb = weight.detach().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            gw = torch.ops.aten.convolution_backward(dyc, x, wb, None, [stride, stride], [pad, pad], [1, 1], False,
                                                     [0, 0], 1, [False, True, False])[1]
            dw = gw.to(weight.dtype)
            CONV3X3_COUNTS["wgrad_miopen"] += 1
        elif dw is not None and not side:
            _native_wgrad_rs(dyc, x, dw, stride, pad)
            if dw.dtype != weight.dtype:
                dw = dw.to(weight.dtype)
        ctx.bn_producer = None
        return dx, dw, None, None, None, None


def _native_wgrad_rs(dyc: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, stride: int, pad: int) -> None:
    """R x S weight gradient into channels_last ``dw``: the 64-channel halo patch kernel where it
    applies, else the det_igemm wgrad ring / gathered gemm_tn."""
    cout, cin, r, s = dw.shape
    out = dw.permute(0, 2, 3, 1).reshape(cout, -1)  # KRSC view of channels_last memory
    assert out.data_ptr() == dw.data_ptr() and out.is_contiguous()
    if not (conv3p_wgrad_ok(cin, cout, r, s, stride, pad) and is_gpu(dyc) and x.data_ptr() % 16 == 0
            and conv3p_wgrad(dyc, x, out)):
        conv_wgrad(dyc, x, out, r, s, stride, pad)
    CONV3X3_COUNTS["wgrad_native"] += 1


def conv_rs(x: torch.Tensor, conv_mod: torch.nn.Conv2d, stats: bool = True, bn_exclusive: bool = False) -> torch.Tensor:
    """``conv_mod(x)`` for bias-free square R x S convs (groups 1, dilation 1, symmetric zero padding)
    on channels_last bf16 CUDA activations with Cin % 64 == 0 and Cout % 64 == 0 (every ResNet 3x3);
    anything else runs the module.  ``bn_exclusive``: this conv is the only autograd consumer of
    ``x``, the output of a fused BatchNorm+ReLU, whose backward partials can then come from the
    stride-1 input-gradient GEMM's epilogue (``FUSE_BN_BWD``)."""
    w = conv_mod.weight
    k = conv_mod.kernel_size
    st = conv_mod.stride
    pd = conv_mod.padding
    ok = (ENABLED and x.device.type == "cuda" and x.dim() == 4 and conv_mod.bias is None and k[0] == k[1]
          and isinstance(pd, tuple) and pd[0] == pd[1] and st[0] == st[1] and conv_mod.dilation == (1, 1)
          and conv_mod.groups == 1 and conv_mod.padding_mode == "zeros" and x.shape[1] % 64 == 0
          and w.shape[0] % 64 == 0 and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0)
    if ok:
        autocast = torch.is_autocast_enabled("cuda")
        if x.dtype != torch.bfloat16 and not (autocast and torch.get_autocast_dtype("cuda") == torch.bfloat16):
            ok = False
    if not ok:
        CONV3X3_COUNTS["fallback"] += 1
        return conv_mod(x)
    CONV3X3_COUNTS["native"] += 1
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    prod = _bn_producer(x) if (bn_exclusive and FUSE_BN_BWD and torch.is_grad_enabled()
                               and (st[0] == 1 or dgrad_s2_ok(x, w, st[0], pd[0]))) else None
    with torch.autocast("cuda", enabled=False):
        return _ConvRS.apply(x, w, int(st[0]), int(pd[0]), stats, prod)
# Stem weight gradient: the det_conv split-M implicit GEMM (True) or MIOpen's NHWC C=4 kernel (False,
# default: 0.49 vs 0.82 ms at batch 512, profiles/r2_stem_microbench.jsonl).  The forward stays native
# (0.64 ms including the BN statistics vs MIOpen 0.70 + a 0.17 ms stats pass).
STEM_NATIVE_WGRAD = False
# Stem weight gradient on the patch kernel (det_igemm.hip stemp_wgrad: dY and the input rows of a
# 256-pixel chunk staged once, transposed operand reads straight from the patch), ahead of both.
STEM_PATCH_WGRAD = os.environ.get("DET_STEM_PATCH_WGRAD", "1") != "0"
# Stem forward on the patch kernel (det_igemm.hip stemp_fwd: the input rows of a 256-pixel chunk
# staged once in LDS, weights resident) instead of det_conv's gathering implicit GEMM (GM_STEM);
# bit-identical outputs, statistics partials per 256 rows.
STEM_PATCH_FWD = os.environ.get("DET_STEM_PATCH_FWD", "1") != "0"
STEM_FWD_COUNTS = {"patch": 0, "gemm": 0}


# ------------------------------------------------------------------------------------------------
# ResNet stem: 7x7 stride-2 pad-3 convolution, 64 filters, over channels padded to 4
# ------------------------------------------------------------------------------------------------
def pack_stem_weight(w: torch.Tensor) -> torch.Tensor:
    """[64, C<=4, 7, 7] -> the [64, 256] bf16 im2col weight det_stem_conv reads: k = r*32 + s*4 + c
    over an 8x8x4 box, zero outside the 7x7xC kernel."""
    co, ci = w.shape[0], w.shape[1]
    wp = torch.zeros(co, 8, 8, 4, dtype=torch.bfloat16, device=w.device)
    wp[:, :7, :7, :ci] = w.detach().permute(0, 2, 3, 1).to(torch.bfloat16)
    return wp.view(co, 256)


def unpack_stem_grad(dwk: torch.Tensor, ci: int) -> torch.Tensor:
    return dwk.view(-1, 8, 8, 4)[:, :7, :7, :ci].permute(0, 3, 1, 2)


def pad_channels4(x: torch.Tensor) -> torch.Tensor:
    """[N, 3, H, W] channels_last -> [N, 4, H, W] channels_last with a zero 4th channel."""
    n, c, h, w = x.shape
    out = torch.empty((n, 4, h, w), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    out[:, c:].zero_()
    out[:, :c] = x
    return out


class _StemConv(torch.autograd.Function):
    """ResNet stem conv as an implicit GEMM on the det_conv MFMA tiles (csrc/det_conv.hip, GM_STEM):
    forward with the stem BatchNorm's statistics in the epilogue (its stats pass over the largest
    activation of the network disappears), weight gradient as a split-M implicit GEMM.  The input
    (the image batch) needs no gradient; when it does, the input gradient comes from MIOpen."""

    @staticmethod
    def forward(ctx, x4, weight, stats):
        n, _, hi, wi = x4.shape
        ho, wo = (hi - 1) // 2 + 1, (wi - 1) // 2 + 1
        m = n * ho * wo
        wk = pack_stem_weight(weight)
        y = torch.empty((n, 64, ho, wo), dtype=torch.bfloat16, device=x4.device, memory_format=torch.channels_last)
        lib = _lib.get_lib()

        def partials(rpb):
            if not stats:
                return None, None, None
            nrb = (m + rpb - 1) // rpb
            pm = torch.empty(nrb, 64, dtype=torch.float32, device=x4.device)
            pq = torch.empty(nrb, 64, dtype=torch.float32, device=x4.device)
            return pm, pq, (pm, pq, rpb)

        rc = -6
        if STEM_PATCH_FWD:
            pm, pq, parts = partials(int(lib.det_stemp_fwd_rows_per_block()))
            rc = lib.det_stemp_fwd(_stream(x4), x4.data_ptr(), wk.data_ptr(), y.data_ptr(), int(m), int(hi), int(wi),
                                   int(ho), int(wo), _ptr(pm), _ptr(pq))
            if rc != -6:
                _lib.check(rc, "stemp_fwd")
                STEM_FWD_COUNTS["patch"] += 1
        if rc == -6:  # the gathering GEMM (any width)
            pm, pq, parts = partials(rows_per_block(64))
            _lib.check(lib.det_stem_conv_fwd(_stream(x4), x4.data_ptr(), wk.data_ptr(), y.data_ptr(), int(m), int(hi),
                                             int(wi), int(ho), int(wo), _ptr(pm), _ptr(pq)), "stem_conv_fwd")
            STEM_FWD_COUNTS["gemm"] += 1
        _attach_partials(y, parts)
        ctx.save_for_backward(x4, weight)
        # the stem BatchNorm may defer its backward apply onto this node (take_pending_apply): the
        # patch wgrad stages it, and the image batch needs no input gradient
        ctx.accepts_bn_apply = is_gpu(x4) and STEM_PATCH_WGRAD and not x4.requires_grad
        ctx.pending_bn_apply = None
        return y

    @staticmethod
    def backward(ctx, dy):
        x4, weight = ctx.saved_tensors
        n, _, hi, wi = x4.shape
        ho, wo = dy.shape[2], dy.shape[3]
        m = n * ho * wo
        pend = take_pending_apply(ctx, dy)
        if pend is not None and (ctx.needs_input_grad[0] or not ctx.needs_input_grad[1]):
            materialize_pending_apply(dy, pend)
            pend = None
        dyc = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        ci = weight.shape[1]
        native_wgrad = False
        if ctx.needs_input_grad[1] and STEM_PATCH_WGRAD:
            # the patch kernel (det_igemm.hip stemp_wgrad): each input row staged once per chunk;
            # with a deferred BN-backward apply, dY = coef . (d, x) is computed while staging
            lib = _lib.get_lib()
            ws = torch.empty(int(lib.det_stemp_wgrad_ws_elems(m)), dtype=torch.float32, device=dy.device)
            dwk = torch.empty(64, 256, dtype=torch.float32, device=dy.device)
            src, bx, coef = (dyc, None, None) if pend is None else pend
            rc = lib.det_stemp_wgrad(_stream(dy), src.data_ptr(), x4.data_ptr(), dwk.data_ptr(), 0, int(m), int(hi),
                                     int(wi), int(ho), int(wo), ws.data_ptr(), 1.0, _ptr(bx), _ptr(coef))
            if rc != -6:
                _lib.check(rc, "stemp_wgrad")
                dw = unpack_stem_grad(dwk, ci).to(weight.dtype).contiguous(memory_format=torch.channels_last)
                native_wgrad = True
                FUSED_COUNTS["stem_wgrad_patch"] += 1
                if pend is not None:
                    BN_APPLY_COUNTS["in_gemm"] += 1
            elif pend is not None:  # the patch does not fit: the apply is needed in HBM after all
                materialize_pending_apply(dy, pend)
                pend = None
        if not native_wgrad and ctx.needs_input_grad[1] and STEM_NATIVE_WGRAD:
            native_wgrad = True
            lib = _lib.get_lib()
            ws = torch.empty(int(lib.det_stem_conv_wgrad_ws_elems(m)), dtype=torch.float32, device=dy.device)
            dwk = torch.empty(64, 256, dtype=torch.float32, device=dy.device)
            _lib.check(lib.det_stem_conv_wgrad(_stream(dy), dyc.data_ptr(), x4.data_ptr(), dwk.data_ptr(), 0, int(m),
                                               int(hi), int(wi), int(ho), int(wo), ws.data_ptr(), 1.0),
                       "stem_conv_wgrad")
            dw = unpack_stem_grad(dwk, ci).to(weight.dtype).contiguous(memory_format=torch.channels_last)
        if ctx.needs_input_grad[0] or (ctx.needs_input_grad[1] and not native_wgrad):
            # MIOpen on the 4-channel problem (its NHWC C=4 wgrad kernel beats the C=3 one 1.4x)
            w4 = torch.empty((64, 4, 7, 7), dtype=torch.bfloat16, device=dy.device, memory_format=torch.channels_last)
            w4[:, ci:].zero_()
            w4[:, :ci] = weight.detach().to(torch.bfloat16)
            gx, gw, _ = torch.ops.aten.convolution_backward(
                dyc, x4, w4, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                [bool(ctx.needs_input_grad[0]), bool(ctx.needs_input_grad[1] and not native_wgrad), False])
            dx = gx
            if gw is not None:
                dw = gw[:, :ci].to(weight.dtype).contiguous(memory_format=torch.channels_last)
        return dx, dw, None


def stem_conv(x: torch.Tensor, conv_mod: torch.nn.Conv2d, stats: bool = True) -> torch.Tensor:
    """``conv_mod(x)`` for the ResNet stem (7x7/2, pad 3, 64 filters, no bias) on channels_last bf16
    CUDA images with 3 channels or 4 (a zero 4th channel, as ``u8_normalize(pad4=True)`` emits).
    Anything else runs the module (on the first 3 channels of a padded input)."""
    w = conv_mod.weight
    ok = (ENABLED and x.device.type == "cuda" and x.dim() == 4 and x.shape[1] in (3, 4) and w.shape[1] <= 4
          and conv_mod.bias is None and conv_mod.kernel_size == (7, 7) and conv_mod.stride == (2, 2)
          and conv_mod.padding in ((3, 3), 3) and conv_mod.dilation == (1, 1) and conv_mod.groups == 1
          and w.shape[0] == 64 and conv_mod.padding_mode == "zeros"
          and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0)
    if ok:
        autocast = torch.is_autocast_enabled("cuda")
        if x.dtype != torch.bfloat16 and not (autocast and torch.get_autocast_dtype("cuda") == torch.bfloat16):
            ok = False
    if not ok:
        FUSED_COUNTS["stem_fallback"] += 1
        return conv_mod(x[:, :w.shape[1]] if x.shape[1] > w.shape[1] else x)
    FUSED_COUNTS["stem"] += 1
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    if x.shape[1] == 3:
        x = pad_channels4(x)
    with torch.autocast("cuda", enabled=False):
        return _StemConv.apply(x, w, stats)


def bn_relu_conv1x1(x: torch.Tensor, bn_mod: torch.nn.modules.batchnorm._BatchNorm,
                    conv_mod: torch.nn.Conv2d) -> torch.Tensor:
    """``conv_mod(relu(bn_mod(x)))``.  Training-mode BN on channels_last bf16 CUDA activations feeding a
    bias-free stride-1 1x1 conv takes ``_BNReluConv1x1`` (BN applied in the GEMM prologue, the
    normalised activation never written); anything else runs the two modules."""
    assert getattr(bn_mod, "relu", False), "bn_relu_conv1x1 needs a BatchNormAct2d with relu=True"
    w = conv_mod.weight
    ok = (ENABLED and getattr(bn_mod, "fused", False) and x.device.type == "cuda" and x.dim() == 4
          and x.dtype == torch.bfloat16 and torch.is_grad_enabled() and bn_mod.training and bn_mod.track_running_stats and bn_mod.affine
          and bn_mod.weight.dtype == torch.float32
          and conv_mod.bias is None and conv_mod.kernel_size == (1, 1) and conv_mod.stride == (1, 1)
          and conv_mod.groups == 1 and conv_mod.padding in ((0, 0), 0, "valid")
          and x.shape[1] % 64 == 0 and w.shape[0] % 64 == 0
          and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0
          and not (torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") != torch.bfloat16))
    if not ok:
        FUSED_COUNTS["fallback"] += 1
        return conv1x1(bn_mod(x), conv_mod)
    FUSED_COUNTS["bn_relu_conv1x1"] += 1
    with torch.autocast("cuda", enabled=False):
        return _BNReluConv1x1.apply(x, bn_mod.weight, bn_mod.bias, bn_mod.running_mean, bn_mod.running_var,
                                    bn_mod.num_batches_tracked, bn_mod.momentum, bn_mod.eps, w)


def conv1x1(x: torch.Tensor, conv_mod: torch.nn.Conv2d, stats: bool = True, bn_exclusive: bool = False) -> torch.Tensor:
    """``conv_mod(x)``; takes the native GEMM path for bias-free 1x1 stride-1 convs on channels_last
    bf16 CUDA activations (channels % 64 == 0), else the module itself.  ``bn_exclusive``: the
    caller guarantees this conv is the only autograd consumer of ``x`` (shortcut consumers go
    through the BN link), which allows the BN-backward fusion into the dgrad (``FUSE_BN_BWD``)."""
    w = conv_mod.weight
    ok = (ENABLED and x.device.type == "cuda" and x.dim() == 4 and conv_mod.bias is None
          and conv_mod.kernel_size == (1, 1) and conv_mod.stride == (1, 1) and conv_mod.groups == 1
          and conv_mod.padding in ((0, 0), 0, "valid") and x.shape[1] % 64 == 0 and w.shape[0] % 64 == 0
          and x.is_contiguous(memory_format=torch.channels_last))
    if ok:
        autocast = torch.is_autocast_enabled("cuda")
        if x.dtype != torch.bfloat16 and not (autocast and torch.get_autocast_dtype("cuda") == torch.bfloat16):
            ok = False
    pend = getattr(x, "_det_fwd_apply", None)
    # (the det_igemm-routed shapes keep det_igemm + the separate apply: staging the apply in
    # gemm_nt there measured 0.5 ms/step slower, profiles/r3_bench_resnet50_defer_fwd_apply.jsonl)
    if pend is not None and not (ok and x.dtype == torch.bfloat16 and w.shape[0] % 64 == 0
                                 and (x.shape[1], w.shape[0]) not in IGEMM_FWD_1X1):
        materialize_fwd_apply(x)  # this conv cannot stage the producer's BN apply itself
        pend = None
    if not ok:
        COUNTS["fallback"] += 1
        return conv_mod(x)
    COUNTS["native"] += 1
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    if pend is not None:
        x._det_fwd_apply = None
    prod = _bn_producer(x) if (bn_exclusive and FUSE_BN_BWD and torch.is_grad_enabled()) else None
    with torch.autocast("cuda", enabled=False):
        return _Conv1x1.apply(x, w, stats, prod, pend)


# ------------------------------------------------------------------------------------------------
# projection shortcut: 1x1 conv, stride 1 or 2 (ResNet downsample)
# ------------------------------------------------------------------------------------------------
# Native projection shortcuts (hparam-free A/B switch): forward on the det_igemm implicit GEMM /
# det_conv gemm_nt with the downsample BN's statistics in the epilogue, input gradient as a 1x1 GEMM
# on the output grid (a stride-2 conv's gradient stays on its stride-2 grid, ``StridedGrad``),
# weight gradient on det_conv's gathered gemm_tn.  Off: MIOpen conv + a separate statistics pass.
NATIVE_SHORTCUT = os.environ.get("DET_NATIVE_SHORTCUT", "1") != "0"
# stride-2 forward tile configuration per (Cin, Cout); default cfg 8 where Cout % 256 == 0
# (profiles/r3_igemm_cfgs_1x1.jsonl: the fastest det_igemm tile on all three ResNet-50 stride-2
# projections), else the automatic choice
SHORTCUT_S2_CFG = {}
SHORTCUT_COUNTS = {"native": 0, "fallback": 0}


def shortcut_native_ok(x: torch.Tensor, conv_mod: torch.nn.Conv2d) -> bool:
    w = conv_mod.weight
    return (NATIVE_SHORTCUT and ENABLED and x.device.type == "cuda" and x.dim() == 4 and conv_mod.bias is None
            and conv_mod.kernel_size == (1, 1) and conv_mod.stride in ((1, 1), (2, 2)) and conv_mod.groups == 1
            and conv_mod.padding in ((0, 0), 0, "valid") and conv_mod.dilation == (1, 1)
            and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.shape[1] % 64 == 0
            and w.shape[0] % 64 == 0 and x.is_contiguous(memory_format=torch.channels_last)
            and x.data_ptr() % 16 == 0 and not torch.is_autocast_enabled("cuda"))


class _Shortcut1x1(torch.autograd.Function):
    """``conv2d(x, w, stride)`` of a 1x1 projection shortcut (stride 1 or 2) on channels_last bf16.

    ``link``: ``x`` is the output of a fused training BN that also feeds the block's conv1; the input
    gradient then goes to that producer's backward (``link.extra_dy``, summed in its kernels -- for
    stride 2 read on the stride-2 grid by the fused dgrad epilogue) and autograd gets None for ``x``
    (reference behaviour: norm._LinkedConv).  Without a link the gradient returns to autograd at
    full resolution."""

    @staticmethod
    def forward(ctx, x, weight, stride, stats, link):
        n, c, h, w_ = x.shape
        cout = weight.shape[0]
        wk = weight.reshape(cout, c)
        wk = (wk if wk.dtype == torch.bfloat16 else wk.to(torch.bfloat16)).contiguous()  # fp32 weights (conv2d_native)
        if stride == 2:
            cfg = SHORTCUT_S2_CFG.get((c, cout), 8 if cout % 256 == 0 else 0)  # cfg 8: 256-wide N tiles
            y, parts = igemm_conv(x, weight, stride=2, stats=stats, w_krsc=wk, cfg=cfg)
        elif (c, cout) in IGEMM_FWD_1X1:
            y, parts = igemm_conv(x, weight, stats=stats, w_krsc=wk, cfg=IGEMM_FWD_1X1[(c, cout)])
        else:
            y2, parts = conv1x1_nt(x.permute(0, 2, 3, 1).reshape(-1, c), wk, stats=stats)
            y = y2.view(n, h, w_, cout).permute(0, 3, 1, 2)
        _attach_partials(y, parts)
        ctx.save_for_backward(x, weight)
        ctx.stride = stride
        ctx.link = link
        if link is not None:
            link.expects_extra = True  # a fused dgrad into the producer must wait for this gradient
        # the shortcut BN may defer its backward apply onto this node (take_pending_apply): the input
        # gradient GEMM stages it (ABN) and writes it for the weight gradient
        ctx.accepts_bn_apply = DGRAD_BT and is_gpu(x)
        ctx.pending_bn_apply = None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        n, c, h, w_ = x.shape
        cout, ho, wo = dy.shape[1], dy.shape[2], dy.shape[3]
        st = ctx.stride
        g = (ho, wo, h, w_) if st == 2 else None
        link, ctx.link = ctx.link, None
        pend = take_pending_apply(ctx, dy)
        if pend is not None and not ((ctx.needs_input_grad[0] or link is not None) and dy.dtype == torch.bfloat16
                                     and dy.is_contiguous(memory_format=torch.channels_last)):
            materialize_pending_apply(dy, pend)
            pend = None
        dy2 = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1).reshape(-1, cout)
        dx = None
        dw, side = _wgrad_target(weight, ctx.needs_input_grad[1], is_gpu(dy2), dy2.numel())
        if side and pend is None:  # independent of the dgrad: fork before it
            with side_work(True, dy2, x):
                _shortcut_wgrad(dy2, x, dw, st, g)
            side = None
        if ctx.needs_input_grad[0] or link is not None:
            w2 = weight.reshape(cout, c)
            w2 = (w2 if w2.dtype == torch.bfloat16 else w2.to(torch.bfloat16)).contiguous()
            abn = None
            if pend is not None:  # dY = the deferred BN apply, staged by the dgrad and written into dy2
                d, bx, coef = pend
                abn = (d.permute(0, 2, 3, 1).reshape(-1, cout), bx, coef, dy2)
                BN_APPLY_COUNTS["in_gemm"] += 1
            dxs = dgrad_1x1(dy2, w2, abn).view(n, ho, wo, c).permute(0, 3, 1, 2)  # on the output grid
            extra = StridedGrad(dxs, g) if st == 2 else dxs
            if link is not None:
                from determined_1_amd.ops.norm import hand_linked_grad

                hand_linked_grad(link, extra)
            else:
                dx = full_res_grad(extra)
        if dw is not None and side is not None:
            with side_work(side, dy2, x):
                _shortcut_wgrad(dy2, x, dw, st, g)
            if dw.dtype != weight.dtype:
                dw = dw.to(weight.dtype)
        return dx, dw, None, None, None


def _shortcut_wgrad(dy2: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, st: int, g: Optional[Gather]) -> None:
    n, c = x.shape[0], x.shape[1]
    cout = dw.shape[0]
    if st == 2 and WGRAD_RING and int(_lib.get_lib().det_igemm_wgrad_ws_elems(dy2.shape[0], cout, c, 0)) > 0:
        # stride 2: the ring's strided im2col beats the gathered gemm_tn on all three ResNet-50
        # projections (0.209 / 0.185 / 0.243 vs 0.228 / 0.208 / 0.316 ms,
        # profiles/r3_shortcut_microbench.jsonl); stride 1 stays on gemm_tn (0.188 vs 0.243)
        ho, wo = g[0], g[1]
        dyc = dy2.view(n, ho, wo, cout).permute(0, 3, 1, 2)
        conv_wgrad(dyc, x, dw.view(cout, c), 1, 1, 2, 0)
    else:
        conv1x1_wgrad(dy2, x.permute(0, 2, 3, 1).reshape(-1, c), dw.view(cout, c), gather=g)


def shortcut_conv1x1(x: torch.Tensor, conv_mod: torch.nn.Conv2d, link=None, stats: bool = True) -> torch.Tensor:
    """Projection-shortcut conv on the native path (``shortcut_native_ok`` must hold)."""
    SHORTCUT_COUNTS["native"] += 1
    return _Shortcut1x1.apply(x, conv_mod.weight, int(conv_mod.stride[0]), stats, link)


# ------------------------------------------------------------------------------------------------
# generic conv2d on the native kernels (detection backbones, FPN)
# ------------------------------------------------------------------------------------------------
# The R50-FPN detectors (Faster / Mask R-CNN, RetinaNet, DETR) run the same ResNet-50 convolution
# shapes as the benchmark, at batch 2 and detection image sizes, without training BatchNorm (frozen,
# folded into the weight and a bias).  ``conv2d_native`` routes a bias-free conv2d to the kernels
# the ResNet trial uses -- 1x1 stride 1 (det_conv gemm_nt / det_igemm), 1x1 stride 2 (det_igemm
# gather), R x S stride 1 / 2 (det_igemm implicit GEMM forward and input gradient, ring / halo-patch
# weight gradient), the 7x7/2 stem (det_conv GM_STEM / patch kernel) -- with the BatchNorm
# statistics epilogues off.  Shapes the tiles do not cover (channels not multiples of 64: the RPN
# / box heads) return None and stay on the library conv.  DET_NATIVE_CONV2D=0 turns it off (A/B).
NATIVE_CONV2D = os.environ.get("DET_NATIVE_CONV2D", "1") != "0"
CONV2D_COUNTS = {"native": 0, "fallback": 0}


def conv2d_native(x: torch.Tensor, weight: torch.Tensor, stride: int = 1, pad: int = 0) -> Optional[torch.Tensor]:
    """``F.conv2d(x, weight, None, stride, pad)`` on the native kernels, or None when not covered
    (CPU, non-channels_last input, fp32 without bf16 autocast, unsupported shape)."""
    if not (NATIVE_CONV2D and ENABLED and x.device.type == "cuda" and x.dim() == 4 and weight.dim() == 4):
        return None
    cout, cin, r, s = weight.shape
    bf = x.dtype == torch.bfloat16 or (torch.is_autocast_enabled("cuda")
                                       and torch.get_autocast_dtype("cuda") == torch.bfloat16)
    if not bf or not x.is_contiguous(memory_format=torch.channels_last) or x.data_ptr() % 16 != 0 or \
            x.shape[1] != cin or x.numel() >= (1 << 31):
        CONV2D_COUNTS["fallback"] += 1
        return None
    kind = None
    if r == s == 1 and pad == 0 and cin % 64 == 0 and cout % 64 == 0 and stride in (1, 2):
        kind = "1x1"
    elif r == s and r in (3, 5) and pad == (r - 1) // 2 and stride in (1, 2) and cin % 64 == 0 and cout % 64 == 0:
        kind = "rs"
    elif r == s == 7 and stride == 2 and pad == 3 and cin in (3, 4) and cout == 64:
        kind = "stem"
    if kind is None:
        CONV2D_COUNTS["fallback"] += 1
        return None
    CONV2D_COUNTS["native"] += 1
    xb = x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16)
    with torch.autocast("cuda", enabled=False):
        if kind == "1x1":
            if stride == 1:
                return _Conv1x1.apply(xb, weight, False, None, None)
            return _Shortcut1x1.apply(xb, weight, 2, False, None)
        if kind == "rs":
            return _ConvRS.apply(xb, weight, int(stride), int(pad), False, None)
        return _StemConv.apply(pad_channels4(xb) if cin == 3 else xb, weight, False)


def conv2d_module(x: torch.Tensor, conv_mod: torch.nn.Conv2d, fallback=None) -> torch.Tensor:
    """``conv_mod(x)`` with the convolution on the native kernels where ``conv2d_native`` covers it
    (square kernel, symmetric zero padding, groups 1, dilation 1); the bias is added after.
    ``fallback`` (default ``conv_mod``) runs the uncovered cases."""
    st, pd = conv_mod.stride, conv_mod.padding
    if isinstance(pd, tuple) and st[0] == st[1] and pd[0] == pd[1] and conv_mod.groups == 1 and \
            conv_mod.dilation == (1, 1) and conv_mod.padding_mode == "zeros":
        y = conv2d_native(x, conv_mod.weight, int(st[0]), int(pd[0]))
        if y is not None:
            if conv_mod.bias is not None:
                y = y + conv_mod.bias.to(y.dtype).view(1, -1, 1, 1)
            return y
    return fallback(x) if fallback is not None else conv_mod(x)
