"""Fused transformer-encoder ops on the ``det_transformer.hip`` kernels.

    linear(x, W, b)                                   y = x W^T + b, bias grad by det_tf_colsum
    linear_gelu(x, W, b[, approximate])               a = gelu(x W^T + b), bias grad fused in gelu bwd
    linear_dropout_add_layernorm(x, W, b, r, g, be)   y = LN(dropout(x W^T + b) + r)
    layer_norm(x, g, be)                              y = LN(x)

GEMMs run on hipBLASLt through ``csrc/det_blaslt.hip`` (one cached descriptor / layout / algorithm
plan per shape, the bias in the library epilogue, beta = 1 for accumulated gradients: ~15 us of host
time per call against 21-26 through ``torch.mm`` / ``addmm``, BERT eager +13-15 %), or on the
hand-written MFMA tiles of ``det_conv.hip`` (``DET_NATIVE_LINEAR``: by default the forward and input
gradient of small weights; forward with the bias in the epilogue, input gradient against the weight
as stored, split-M weight gradient); everything between them is one HIP
pass per direction, and every Linear's bias gradient is produced inside the kernel that already
reads the gradient (LayerNorm bwd, GELU bwd) instead of a separate reduction.  Dropout masks are
regenerated from a Philox (seed, offset) pair in the backward pass rather than stored.

CPU tensors, and GPU layouts the kernels do not cover (fp16, hidden > 8192, hidden % 8 != 0),
run the plain PyTorch composite, which is also the numerics reference of the GPU tests; GPU
fallbacks are counted in ``FALLBACKS`` so benchmarks can assert the native path ran.
"""
import ctypes
import os
from typing import Any, Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from determined_1_amd.ops import _lib
from determined_1_amd.ops.arena import landing_buffer

FALLBACKS = {"count": 0}
_DT = {torch.float32: 0, torch.bfloat16: 1}
_MAX_H = 8192  # det_tf_ln_max_hidden() (workgroup-per-row kernels above 2048, e.g. ALBERT-xxlarge)
# Philox (seed, offset) stream of the native dropout kernels (LayerNorm + residual dropout,
# attention dropout).  Part of the trial's RNG state: reset when the trial seeds its RNGs and saved /
# restored with its checkpoints (pytorch/_trial.py), so a resumed trial draws the masks an
# uninterrupted one would.  The seed is taken lazily from torch's at the first call.
_RNG = {"seed": None, "offset": 1}
_MASK64 = 0xFFFFFFFFFFFFFFFF


def _stream(t: torch.Tensor) -> int:
    return torch._C._cuda_getCurrentRawStream(t.device.index)


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def next_rng() -> Tuple[int, int]:
    """(seed, offset) of the next dropout call: the seed follows the trial's torch seed, the offset
    is unique per call, so masks are reproducible run to run and across checkpoint/restore."""
    if _RNG["seed"] is None:
        _RNG["seed"] = torch.initial_seed() & _MASK64
    off = _RNG["offset"]
    _RNG["offset"] = off + 1
    return _RNG["seed"], off


_RNG_BASE = {}  # type: Dict[int, torch.Tensor]  # device index -> int32 [1] offset counter


def rng_base(device: torch.device) -> int:
    """Device pointer of the dropout offset counter the kernels add to their captured (seed, offset)
    (det_transformer.hip Rng::obase, det_attention.hip Args::rng_base)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    t = _RNG_BASE.get(idx)
    if t is None:
        t = _RNG_BASE[idx] = torch.zeros(1, dtype=torch.int32, device=torch.device("cuda", idx))
    return t.data_ptr()


def bump_rng_base() -> None:
    """Advance every device's dropout offset counter on the current stream.  A captured train step
    starts with this, so each hipGraph replay draws new masks from the same captured arguments."""
    lib = _lib.get_lib()
    for idx, t in _RNG_BASE.items():
        _lib.check(lib.det_tf_rng_bump(torch.cuda.current_stream(torch.device("cuda", idx)).cuda_stream,
                                       t.data_ptr()), "det_tf_rng_bump")


def reset_rng(seed: Optional[int] = None) -> None:
    """Start a new stream (the trial controller calls this when it seeds torch)."""
    _RNG["seed"] = None if seed is None else int(seed) & _MASK64
    _RNG["offset"] = 1


def rng_state() -> Dict[str, Any]:
    return {"seed": _RNG["seed"], "offset": _RNG["offset"],
            "base": {idx: int(t.item()) for idx, t in _RNG_BASE.items()}}


def set_rng_state(state: Dict[str, Any]) -> None:
    _RNG["seed"] = state.get("seed")
    _RNG["offset"] = int(state.get("offset", 1))
    for idx, v in (state.get("base") or {}).items():
        if torch.cuda.is_available() and int(idx) < torch.cuda.device_count():
            rng_base(torch.device("cuda", int(idx)))
            _RNG_BASE[int(idx)].fill_(int(v))


def rng_calls() -> int:
    """Native dropout calls so far."""
    return _RNG["offset"] - 1


def _native(*ts: Optional[torch.Tensor], width: int, max_width: Optional[int] = None) -> bool:
    dev = [t for t in ts if t is not None]
    if not dev or dev[0].device.type != "cuda":
        return False
    dt = dev[0].dtype
    ok = dt in _DT and all(t.dtype == dt and t.device == dev[0].device for t in dev) and width % 8 == 0
    if max_width is not None:
        ok = ok and width <= max_width
    if not ok:
        FALLBACKS["count"] += 1
    return ok


def _autocast(*ts: Optional[torch.Tensor]):
    """Under autocast run in the autocast dtype (what F.linear would do) with autocast off."""
    if torch.is_autocast_enabled("cuda") and any(t is not None and t.is_cuda for t in ts):
        dt = torch.get_autocast_dtype("cuda")
        return [t.to(dt) if t is not None and t.is_floating_point() else t for t in ts], True
    return list(ts), False


class SharedWeightGrads:
    """Weight gradients of layers applied several times in one forward (ALBERT's shared layer).

    Autograd would compute one dW per use and sum them in its input buffer: an elementwise add of
    the whole weight per extra use (11 x 201M elements per ALBERT-xxlarge step, 6 % of the step
    in profiles/r1_albert_xxlarge_bs8_o2_per_step.txt).  Instead the first backward use writes dW
    with a GEMM, later uses accumulate into it with ``addmm_`` (hipBLASLt beta = 1, no extra pass)
    and only the last use hands the buffer to autograd; the other uses return None.
    Create one per forward pass (``track`` counts the uses of each weight)."""

    def __init__(self) -> None:
        self._state = {}  # id(weight) -> [remaining uses, buffer]

    def track(self, weight: torch.Tensor) -> "SharedWeightGrads":
        st = self._state.setdefault(id(weight), [0, None])
        st[0] += 1
        return self

    def accumulate(self, weight: torch.Tensor, dz: torch.Tensor, x2: torch.Tensor) -> Optional[torch.Tensor]:
        st = self._state[id(weight)]
        if st[1] is None:
            st[1] = _weight_grad(weight, dz, x2)[0]
        elif _bl_ok(dz, x2, st[1]):
            _bl_wgrad(dz, x2, st[1].view(dz.shape[1], x2.shape[1]), beta=1.0)
        else:
            st[1].addmm_(dz.t(), x2)
        st[0] -= 1
        if st[0] > 0:
            return None
        out, st[1] = st[1], None
        return out


# Dense layers on the hand-written det_conv.hip GEMMs instead of the vendor BLAS.
#   "1": every pass;  "0": none;  "auto" (default): the forward and input-gradient GEMMs of small
#   weights (<= NATIVE_AUTO_MAX_WEIGHT elements), where the tiles beat the (tuned) library: BERT-base's
#   768x768 attention output at 4608 tokens, forward 14.1 vs 23.9 us, input gradient 13.4 vs 26.5 us;
#   the 768x2304 / 768x3072 layers and every weight gradient stay on the library, which wins there
#   (profiles/r5_bert_linear_shapes.json, scripts/bench_linear_shapes.py).
NATIVE_LINEAR = os.environ.get("DET_NATIVE_LINEAR", "auto")
NATIVE_AUTO_MAX_WEIGHT = 1 << 20
LINEAR_COUNTS = {"native_fwd": 0, "native_dgrad": 0, "native_wgrad": 0, "gemm8_gelu_fwd": 0}

# The FFN-in Linear + GELU forward on the hand-written eight-phase GEMM (ops/csrc/det_gemm8.hip) with
# the GELU in its epilogue (pre-activation and activation written from one C tile) instead of the
# vendor GEMM plus a separate GELU pass; for outputs of at least GEMM8_MIN_ELEMS elements (the tile
# is 256 x 256).  Opt-in (DET_GEMM8_FFN=1): measured 0.4-1.1 % slower than hipBLASLt + the GELU pass
# in the BERT graph step (1,462-1,465 vs 1,471-1,479 examples/s, profiles/r6_bert_gemm8_ffn_ab.jsonl)
# -- the 4608 x 3072 x 768 GEMM is 8 % slower on the hand-written tile (r6_gemm8_vs_hipblaslt.jsonl).
GEMM8_FFN = os.environ.get("DET_GEMM8_FFN", "0") == "1"
GEMM8_MIN_ELEMS = 1 << 22


def _gemm8_gelu(x2: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], approx: bool):
    """(z, gelu(z)) from one det_gemm8 launch, or None when the shape / dtypes do not fit."""
    if not (GEMM8_FFN and x2.is_cuda and x2.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16
            and x2.shape[0] * weight.shape[0] >= GEMM8_MIN_ELEMS
            and (bias is None or (bias.dtype in (torch.bfloat16, torch.float32) and bias.is_contiguous()))):
        return None
    from determined_1_amd.ops import gemm8 as _g8

    if not _g8.supported(x2, weight):
        return None
    z = torch.empty(x2.shape[0], weight.shape[0], dtype=torch.bfloat16, device=x2.device)
    a = torch.empty_like(z)
    _g8.gemm8(x2, weight, bias=bias, out=z, gelu_out=a, gelu=2 if approx else 1)
    LINEAR_COUNTS["gemm8_gelu_fwd"] += 1
    return z, a


def _native_linear(x2: torch.Tensor, weight: torch.Tensor, wgrad: bool = False) -> bool:
    mode = NATIVE_LINEAR
    if mode is True or mode == "1":
        on = True
    elif mode == "auto":
        on = not wgrad and weight.numel() <= NATIVE_AUTO_MAX_WEIGHT
    else:
        on = False
    return (on and x2.is_cuda and x2.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16
            and x2.dim() == 2 and x2.is_contiguous() and weight.is_contiguous() and weight.shape[0] % 64 == 0
            and weight.shape[1] % 64 == 0 and x2.data_ptr() % 16 == 0 and weight.data_ptr() % 16 == 0)


# Library GEMMs through ops/csrc/det_blaslt.hip: hipBLASLt with a cached plan per shape instead of
# torch.mm / addmm (21-26 us of host time per call in the BERT eager step, r5s32); DET_BLASLT=0 off.
BLASLT = os.environ.get("DET_BLASLT", "1") != "0"
_BL = {"ready": None, "ws": {}}  # type: Dict[str, Any]
_BL_WS_BYTES = 32 << 20
_BL_DT = {torch.bfloat16: 1, torch.float32: 0}


def _bl_ok(*ts: torch.Tensor) -> bool:
    if not BLASLT or not ts[0].is_cuda:
        return False
    dt = ts[0].dtype
    if dt not in _BL_DT or any(t.dtype != dt or not t.is_contiguous() or t.dim() > 2 or t.data_ptr() % 16 for t in ts):
        return False  # the cached plans assume 16-B aligned operands
    ready = _BL["ready"]
    if ready is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "libhipblaslt.so")
        lib = _lib.get_lib()
        ready = _BL["ready"] = os.path.exists(path) and lib.det_blaslt_init(path.encode()) == 0
        _BL["fn"] = lib.det_blaslt_gemm
    if not ready:
        return False
    key = (ts[0].device.index, torch._C._cuda_getCurrentRawStream(ts[0].device.index))
    if key not in _BL["ws"]:
        # one workspace per (device, stream), as torch keeps its BLAS workspaces: GEMMs on two
        # streams (an eager step beside a graph replay, a side stream) never share scratch.  Made
        # inside a capture it comes from that graph's private pool and stays allocated (held here).
        _BL["ws"][key] = torch.empty(_BL_WS_BYTES, dtype=torch.uint8, device=ts[0].device)
    return True


def _bl_gemm(ta: int, tb: int, m: int, n: int, k: int, A: torch.Tensor, lda: int, B: torch.Tensor, ldb: int,
             D: torch.Tensor, ldd: int, bias: Optional[torch.Tensor] = None, beta: float = 0.0,
             bias_grad: bool = False) -> int:
    """Column-major D[m, n] = op(A) op(B) [+ bias per row] [+ beta D] (see det_blaslt.hip); with
    ``bias_grad`` the epilogue instead WRITES bias[n] = sum_k op(B)[k, n] (returns the library code,
    non-zero when no algorithm supports that epilogue, instead of raising)."""
    dev = D.device.index
    stream = torch._C._cuda_getCurrentRawStream(dev)
    rc = _BL["fn"](stream, ta, tb, m, n, k, A.data_ptr(), lda, B.data_ptr(), ldb,
                   D.data_ptr(), ldd, None if bias is None else bias.data_ptr(), beta, _BL_DT[D.dtype],
                   _BL["ws"][(dev, stream)].data_ptr(), _BL_WS_BYTES, 2 if bias_grad else 1)
    if rc != 0 and not bias_grad:
        _lib.check(rc, "det_blaslt_gemm")
    return rc


# Linear bias gradients from the weight-gradient GEMM's epilogue (hipBLASLt BGRADB) instead of a
# two-launch column sum; shapes whose plan has no such algorithm fall back (remembered here).
# Opt-in (DET_BGRAD_EPILOGUE=1): the BERT graph step measured the same either way (1,514-1,527 vs
# 1,516-1,522 examples/s, profiles/r6_bert_bgrad_epilogue_ab.jsonl) -- the epilogue plan's GEMM costs
# what the column sum saved.
BGRAD_EPILOGUE = os.environ.get("DET_BGRAD_EPILOGUE", "0") == "1"
_BGRAD_UNSUPPORTED = set()  # type: set
LINEAR_BGRAD_COUNTS = {"epilogue": 0, "colsum": 0}


def _bl_wgrad(dz: torch.Tensor, x2: torch.Tensor, out: torch.Tensor, beta: float = 0.0,
              db: Optional[torch.Tensor] = None) -> bool:
    """out[N, K] (+)= dz[M, N]^T x2[M, K]; with ``db`` [N] also db = column sums of dz from the
    same GEMM when the library supports it.  Returns whether db was written."""
    M, N = dz.shape
    K = x2.shape[1]
    key = (M, N, K, dz.dtype, beta != 0.0)
    if db is not None and BGRAD_EPILOGUE and key not in _BGRAD_UNSUPPORTED:
        if _bl_gemm(0, 1, K, N, M, x2, K, dz, N, out, K, bias=db, beta=beta, bias_grad=True) == 0:
            LINEAR_BGRAD_COUNTS["epilogue"] += 1
            return True
        _BGRAD_UNSUPPORTED.add(key)
    _bl_gemm(0, 1, K, N, M, x2, K, dz, N, out, K, beta=beta)
    return False


def _weight_grad(weight: torch.Tensor, dz: torch.Tensor, x2: torch.Tensor,
                 db: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, bool]:
    """dW = dz^T x, written straight into the parameter's gradient-arena slot when that is where
    it will land (ops.arena.landing_buffer): no separate landing copy for the largest gradients.
    With ``db``: also the bias gradient from the GEMM epilogue where the library path allows it;
    returns (dW, whether db was written)."""
    buf = landing_buffer(weight) if weight.is_cuda else None
    if _native_linear(x2, weight, wgrad=True) and dz.dtype == torch.bfloat16 and dz.is_contiguous():
        from determined_1_amd.ops.conv import conv1x1_wgrad

        out = buf if (buf is not None and buf.dtype in (torch.bfloat16, torch.float32) and buf.is_contiguous()) \
            else torch.empty(weight.shape, dtype=weight.dtype, device=weight.device)
        conv1x1_wgrad(dz, x2, out.view(weight.shape[0], -1))
        LINEAR_COUNTS["native_wgrad"] += 1
        return out, False
    if _bl_ok(dz, x2):
        out = buf if (buf is not None and buf.dtype == dz.dtype and buf.is_contiguous()) else \
            torch.empty(weight.shape, dtype=dz.dtype, device=dz.device)
        done = _bl_wgrad(dz, x2, out.view(dz.shape[1], x2.shape[1]), db=db)
        return out.view(weight.shape), done
    if buf is not None and buf.dtype == dz.dtype and buf.is_contiguous():
        return torch.mm(dz.t(), x2, out=buf), False
    return dz.t() @ x2, False


def _mm_backward(dz: torch.Tensor, x2: torch.Tensor, weight: torch.Tensor, need_x: bool, need_w: bool,
                 acc: Optional[SharedWeightGrads] = None, dr: Optional[torch.Tensor] = None,
                 db: Optional[torch.Tensor] = None):
    """dr: a gradient of x2 from another use (ResidualGradLink), summed into dx by the GEMM.  db: a
    bias-gradient buffer the weight-gradient GEMM may fill from its epilogue; the third result says
    whether it did."""
    if dr is not None and not need_x:
        raise RuntimeError("a linked residual gradient reached a Linear whose input needs no gradient")
    if need_x and _native_linear(x2, weight) and dz.dtype == torch.bfloat16 and dz.is_contiguous():
        from determined_1_amd.ops.conv import dgrad_1x1

        dx = dgrad_1x1(dz, weight)  # dz [M, N] . W [N, K], the weight read as stored
        LINEAR_COUNTS["native_dgrad"] += 1
        if dr is not None:
            dx = dx.add_(dr)
    elif need_x and dr is not None and dr.dtype == dz.dtype and dr.shape == x2.shape and dr.is_contiguous():
        # dr + dz W: hipBLASLt beta = 1 instead of autograd's separate add
        if _bl_ok(dz, weight, dr):
            M, N = dz.shape
            K = weight.shape[1]
            _bl_gemm(0, 0, K, M, N, weight, K, dz, N, dr, K, beta=1.0)
            dx = dr
        else:
            dx = dr.addmm_(dz, weight)
    elif need_x and _bl_ok(dz, weight):
        M, N = dz.shape
        K = weight.shape[1]
        dx = torch.empty(M, K, dtype=dz.dtype, device=dz.device)
        _bl_gemm(0, 0, K, M, N, weight, K, dz, N, dx, K)
        if dr is not None:  # a linked residual gradient the beta = 1 branch could not take (layout)
            dx.add_(dr.reshape(dx.shape))
    else:
        dx = dz @ weight if need_x else None
        if dr is not None:
            dx = dx + dr.view(dx.shape)
    dw = None
    db_done = False
    if need_w:
        if acc is not None:
            dw = acc.accumulate(weight, dz, x2)
        else:
            dw, db_done = _weight_grad(weight, dz, x2, db)
    return dx, dw, db_done


def _track(acc: Optional[SharedWeightGrads], weight: torch.Tensor) -> Optional[SharedWeightGrads]:
    if acc is None or not (torch.is_grad_enabled() and weight.requires_grad):
        return None
    return acc.track(weight)


def _addmm(x2: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    if _native_linear(x2, weight) and (bias is None or (bias.dtype == torch.bfloat16 and bias.is_contiguous())):
        y = torch.empty(x2.shape[0], weight.shape[0], dtype=torch.bfloat16, device=x2.device)
        _lib.check(_lib.get_lib().det_linear_fwd(_stream(x2), x2.data_ptr(), weight.data_ptr(), _ptr(bias), y.data_ptr(),
                                                 int(x2.shape[0]), int(weight.shape[0]), int(x2.shape[1])),
                   "det_linear_fwd")
        LINEAR_COUNTS["native_fwd"] += 1
        return y
    if _bl_ok(x2, weight) and (bias is None or (bias.dtype == x2.dtype and bias.is_contiguous())):
        M, K = x2.shape
        N = weight.shape[0]
        y = torch.empty(M, N, dtype=x2.dtype, device=x2.device)
        _bl_gemm(1, 0, N, M, K, weight, K, x2, K, y, N, bias=bias)
        return y
    return torch.addmm(bias, x2, weight.t()) if bias is not None else x2 @ weight.t()


class ResidualGradLink:
    """A tensor read by a Linear and again, later in the forward, as the residual of
    ``linear_dropout_add_layernorm`` (a BERT layer's input and its attention output).  Autograd
    computes the two input gradients separately and adds them: one elementwise pass over [rows, H]
    per use, 24 per BERT-base step (``CUDAFunctor_add`` in profiles/r4_bert_steady.txt).  With a
    link, the LayerNorm backward -- which runs first -- parks its residual gradient here and the
    Linear's input-gradient GEMM accumulates onto it (hipBLASLt beta = 1).  The Linear arms the link
    with its input; the LayerNorm only parks a gradient when its residual is that same tensor."""

    __slots__ = ("x", "dr")

    def __init__(self) -> None:
        self.x = None  # type: Optional[torch.Tensor]
        self.dr = None  # type: Optional[torch.Tensor]

    def take(self) -> Optional[torch.Tensor]:
        dr, self.dr = self.dr, None
        return dr


def _arm(link: Optional[ResidualGradLink], x: torch.Tensor) -> Optional[ResidualGradLink]:
    if link is None or not (torch.is_grad_enabled() and x.requires_grad):
        return None
    link.x, link.dr = x, None
    return link


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, acc, link=None):
        x2 = x.reshape(-1, x.shape[-1])
        y = _addmm(x2, weight, bias)
        ctx.acc = acc
        ctx.link = link
        ctx.save_for_backward(x2, weight)
        ctx.has_bias = bias is not None
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        dy2 = dy.reshape(-1, weight.shape[0]).contiguous()
        dr = ctx.link.take() if ctx.link is not None else None
        want_db = ctx.has_bias and ctx.needs_input_grad[2]
        db = torch.empty(dy2.shape[1], dtype=dy2.dtype, device=dy2.device) if want_db else None
        dx, dw, db_done = _mm_backward(dy2, x2, weight, ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.acc, dr,
                                       db=db)
        if want_db and not db_done:
            lib = _lib.get_lib()
            rows, C = dy2.shape
            ws = torch.empty(int(lib.det_tf_col_ws_elems(rows, C)), dtype=torch.float32, device=dy2.device)
            _lib.check(lib.det_tf_colsum(_stream(dy2), _DT[dy2.dtype], dy2.data_ptr(), rows, C, db.data_ptr(),
                                         ws.data_ptr()), "det_tf_colsum")
            LINEAR_BGRAD_COUNTS["colsum"] += 1
        return (dx.view(ctx.xshape) if dx is not None else None), dw, db, None, None


class _LinearGELU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, approx, acc, link=None):
        x2 = x.reshape(-1, x.shape[-1])
        ctx.link = link
        fused = None if _native_linear(x2, weight) else _gemm8_gelu(x2, weight, bias, bool(approx))
        if fused is not None:
            z, a = fused
        else:
            z = _addmm(x2, weight, bias)
            a = torch.empty_like(z)
            lib = _lib.get_lib()
            _lib.check(lib.det_tf_gelu_fwd(_stream(z), _DT[z.dtype], z.data_ptr(), a.data_ptr(), z.numel(),
                                           int(approx)), "det_tf_gelu_fwd")
        ctx.approx = int(approx)
        ctx.acc = acc
        ctx.save_for_backward(x2, weight, z)
        ctx.has_bias = bias is not None
        ctx.xshape = x.shape
        return a.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, da):
        x2, weight, z = ctx.saved_tensors
        rows, C = z.shape
        da2 = da.reshape(rows, C).contiguous()
        lib = _lib.get_lib()
        dz = torch.empty_like(z)
        db = torch.empty(C, dtype=z.dtype, device=z.device) if ctx.has_bias and ctx.needs_input_grad[2] else None
        ws = torch.empty(int(lib.det_tf_col_ws_elems(rows, C)) if db is not None else 1, dtype=torch.float32,
                         device=z.device)
        _lib.check(lib.det_tf_gelu_bwd(_stream(z), _DT[z.dtype], da2.data_ptr(), z.data_ptr(), dz.data_ptr(), rows, C,
                                       _ptr(db), ws.data_ptr(), ctx.approx), "det_tf_gelu_bwd")
        dr = ctx.link.take() if ctx.link is not None else None
        dx, dw, _ = _mm_backward(dz, x2, weight, ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.acc, dr)
        return (dx.view(ctx.xshape) if dx is not None else None), dw, db, None, None, None


def _ln_forward(h: torch.Tensor, r: Optional[torch.Tensor], gamma, beta, p: float, eps: float):
    rows, H = h.shape
    lib = _lib.get_lib()
    y = torch.empty_like(h)
    mean = torch.empty(rows, dtype=torch.float32, device=h.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=h.device)
    seed, off = next_rng() if p > 0 else (0, 0)
    _lib.check(lib.det_tf_ln_fwd(_stream(h), _DT[h.dtype], h.data_ptr(), _ptr(r), y.data_ptr(), rows, H,
                                 gamma.data_ptr(), beta.data_ptr(), eps, p, seed, off, mean.data_ptr(),
                                 rstd.data_ptr(), rng_base(h.device) if p > 0 else None), "det_tf_ln_fwd")
    return y, mean, rstd, seed, off


def _ln_backward(ctx, dy, h, r, gamma, mean, rstd, need_dh: bool, need_dr: bool, need_bias: bool):
    rows, H = h.shape
    lib = _lib.get_lib()
    dy2 = dy.reshape(rows, H).contiguous()
    dh = torch.empty_like(h) if need_dh else None
    dr = torch.empty_like(h) if need_dr else None
    dgamma = torch.empty_like(gamma) if ctx.need_gamma else None
    dbeta = torch.empty_like(gamma) if ctx.need_beta else None
    dbias = torch.empty(H, dtype=h.dtype, device=h.device) if need_bias else None
    ws = torch.empty(int(lib.det_tf_ln_ws_elems(rows, H)), dtype=torch.float32, device=h.device)
    _lib.check(lib.det_tf_ln_bwd(_stream(h), _DT[h.dtype], dy2.data_ptr(), h.data_ptr(), _ptr(r), mean.data_ptr(),
                                 rstd.data_ptr(), gamma.data_ptr(), rows, H, ctx.p, ctx.seed, ctx.off, _ptr(dr),
                                 _ptr(dh), _ptr(dgamma), _ptr(dbeta), _ptr(dbias), ws.data_ptr(),
                                 rng_base(h.device) if ctx.p > 0 else None), "det_tf_ln_bwd")
    return dh, dr, dgamma, dbeta, dbias


class _LinearDropAddLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, gamma, beta, p, eps, acc, link=None):
        x2 = x.reshape(-1, x.shape[-1])
        ctx.acc = acc
        # park the residual gradient for the Linear that read this same tensor (ResidualGradLink)
        ctx.link = link if link is not None and link.x is residual else None
        h = _addmm(x2, weight, bias)
        r2 = residual.reshape(h.shape).contiguous()
        y, mean, rstd, ctx.seed, ctx.off = _ln_forward(h, r2, gamma, beta, p, eps)
        ctx.p = p
        ctx.has_bias = bias is not None
        ctx.xshape, ctx.rshape = x.shape, residual.shape
        ctx.need_gamma, ctx.need_beta = ctx.needs_input_grad[4], ctx.needs_input_grad[5]
        ctx.save_for_backward(x2, weight, h, r2, gamma, mean, rstd)
        return y.view(residual.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, h, r2, gamma, mean, rstd = ctx.saved_tensors
        need_h = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        dh, dr, dgamma, dbeta, dbias = _ln_backward(
            ctx, dy, h, r2, gamma, mean, rstd, need_dh=True, need_dr=ctx.needs_input_grad[3],
            need_bias=ctx.has_bias and ctx.needs_input_grad[2])
        if ctx.link is not None and dr is not None:
            ctx.link.dr, dr = dr, None
        dx, dw, _ = (_mm_backward(dh, x2, weight, ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.acc)
                     if need_h else (None, None, False))
        return ((dx.view(ctx.xshape) if dx is not None else None), dw, dbias,
                (dr.view(ctx.rshape) if dr is not None else None), dgamma, dbeta, None, None, None, None)


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        h = x.reshape(-1, x.shape[-1]).contiguous()
        y, mean, rstd, ctx.seed, ctx.off = _ln_forward(h, None, gamma, beta, 0.0, eps)
        ctx.p = 0.0
        ctx.xshape = x.shape
        ctx.need_gamma, ctx.need_beta = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        ctx.save_for_backward(h, gamma, mean, rstd)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        h, gamma, mean, rstd = ctx.saved_tensors
        dh, _, dgamma, dbeta, _ = _ln_backward(ctx, dy, h, None, gamma, mean, rstd, need_dh=ctx.needs_input_grad[0],
                                               need_dr=False, need_bias=False)
        return (dh.view(ctx.xshape) if dh is not None else None), dgamma, dbeta, None


def _split_qkv(qkv: torch.Tensor, nh: int):
    B, S, H3 = qkv.shape
    hd = H3 // 3 // nh
    return qkv.view(B, S, 3, nh, hd).permute(2, 0, 3, 1, 4).unbind(0)  # 3 x [B, nh, S, hd] views


class _AttnParams(ctypes.Structure):
    """Mirror of ``DetAttnParams`` (det_attention.hip)."""
    _fields_ = ([(n, ctypes.c_void_p) for n in ("q", "k", "v", "dout", "out", "dq", "dk", "dv", "lse", "delta",
                                                "kbias", "mbias")]
                + [(n, ctypes.c_int64) for n in ("qsb", "qst", "ksb", "kst", "vsb", "vst", "osb", "ost", "dosb",
                                                 "dost", "dqsb", "dqst", "dksb", "dkst", "dvsb", "dvst", "mbb", "mbh",
                                                 "mbq")]
                + [(n, ctypes.c_int32) for n in ("B", "Lq", "Lk", "nh", "hd", "dtype")]
                + [("p", ctypes.c_float), ("scale", ctypes.c_float), ("seed", ctypes.c_uint64),
                   ("offset", ctypes.c_uint64), ("rng_base", ctypes.c_void_p)])


_ATTN_DT = {torch.bfloat16: 0, torch.float32: 1}


def mfma_attention_supported(Lq: int, head_dim: int, dtype: torch.dtype = torch.bfloat16,
                             Lk: Optional[int] = None) -> bool:
    """Whether ``det_attention.hip`` covers the shape (bf16 head_dim 32/64/128, fp32 32/64, any
    length up to what the LDS tiles allow).  ``DET_ATTN=composite`` forces the PyTorch path."""
    import os

    if os.environ.get("DET_ATTN", "mfma") != "mfma" or dtype not in _ATTN_DT:
        return False
    return bool(_lib.get_lib().det_attn_supported(_ATTN_DT[dtype], head_dim, Lq, Lq if Lk is None else Lk))


def _view_ok(t: torch.Tensor, hd: int) -> bool:
    """[B, L, nh*hd] token-major view the kernels read in place: unit inner stride, 16-B aligned rows."""
    es = t.element_size()
    return (t.dim() == 3 and t.stride(2) == 1 and t.data_ptr() % 16 == 0 and (t.stride(1) * es) % 16 == 0
            and (t.stride(0) * es) % 16 == 0)


def _bias_args(bias: Optional[torch.Tensor], B: int, nh: int, Lq: int, Lk: int):
    """Split an additive / boolean SDPA mask into the kernels' per-key row [B, Lk] (padding masks)
    or a strided full bias (element (b, h, q, k) at b*sb + h*sh + q*sq + k).  -> (kbias, mbias, strides)"""
    if bias is None:
        return None, None, (0, 0, 0)
    if bias.dtype == torch.bool:  # SDPA semantics: True = attend
        bias = torch.zeros(bias.shape, dtype=torch.float32, device=bias.device).masked_fill_(~bias, float("-inf"))
    bias = bias.float()
    while bias.dim() < 4:
        bias = bias.unsqueeze(0)
    if bias.shape[1] == 1 and bias.shape[2] == 1:  # [B|1, 1, 1, Lk]: a per-key row
        return bias.reshape(bias.shape[0], Lk).expand(B, Lk).contiguous(), None, (0, 0, 0)
    full = bias.expand(B, nh, Lq, Lk)
    if full.stride(3) != 1:
        full = bias.contiguous().expand(B, nh, Lq, Lk)
    return None, full, (full.stride(0), full.stride(1), full.stride(2))


def _attn_params(q, k, v, nh: int, kbias, mbias, mstrides, p: float, scale: float) -> _AttnParams:
    B, Lq, H = q.shape
    P = _AttnParams()
    P.q, P.k, P.v = q.data_ptr(), k.data_ptr(), v.data_ptr()
    P.qsb, P.qst = q.stride(0), q.stride(1)
    P.ksb, P.kst = k.stride(0), k.stride(1)
    P.vsb, P.vst = v.stride(0), v.stride(1)
    P.kbias, P.mbias = _ptr(kbias), _ptr(mbias)
    P.mbb, P.mbh, P.mbq = mstrides
    P.B, P.Lq, P.Lk, P.nh, P.hd, P.dtype = B, Lq, k.shape[1], nh, H // nh, _ATTN_DT[q.dtype]
    P.p, P.scale = p, scale
    return P


def _attn_forward(q, k, v, nh, kbias, mbias, mstrides, p, scale):
    B, Lq, H = q.shape
    out = torch.empty(B, Lq, H, dtype=q.dtype, device=q.device)
    lse = torch.empty(B, nh, Lq, dtype=torch.float32, device=q.device)
    seed, off = next_rng() if p > 0 else (0, 0)
    P = _attn_params(q, k, v, nh, kbias, mbias, mstrides, p, scale)
    P.out, P.lse, P.osb, P.ost = out.data_ptr(), lse.data_ptr(), out.stride(0), out.stride(1)
    P.seed, P.offset = seed, off
    P.rng_base = rng_base(q.device) if p > 0 else None
    _lib.check(_lib.get_lib().det_attn_forward(_stream(q), ctypes.byref(P)), "det_attn_forward")
    return out, lse, seed, off


def _attn_backward(ctx, dout, q, k, v, out, lse, kbias, mbias, dq, dk, dv):
    dout = dout if _view_ok(dout, 1) else dout.contiguous()
    P = _attn_params(q, k, v, ctx.nh, kbias, mbias, ctx.mstrides, ctx.p, ctx.scale)
    delta = torch.empty_like(lse)
    P.out, P.lse, P.delta, P.dout = out.data_ptr(), lse.data_ptr(), delta.data_ptr(), dout.data_ptr()
    P.osb, P.ost, P.dosb, P.dost = out.stride(0), out.stride(1), dout.stride(0), dout.stride(1)
    P.dq, P.dk, P.dv = dq.data_ptr(), dk.data_ptr(), dv.data_ptr()
    P.dqsb, P.dqst, P.dksb, P.dkst, P.dvsb, P.dvst = (dq.stride(0), dq.stride(1), dk.stride(0), dk.stride(1),
                                                      dv.stride(0), dv.stride(1))
    P.seed, P.offset = ctx.seed, ctx.off
    P.rng_base = rng_base(q.device) if ctx.p > 0 else None
    _lib.check(_lib.get_lib().det_attn_backward(_stream(q), ctypes.byref(P)), "det_attn_backward")


class _PackedQKVAttention(torch.autograd.Function):
    """``det_attention.hip`` on the fused [B, S, 3H] QKV GEMM output: Q/K/V read in place as strided
    views, dQ/dK/dV written straight into the [B, S, 3H] gradient (no split/pack copies); dropout
    masks are regenerated from (seed, offset) in the backward."""

    @staticmethod
    def forward(ctx, qkv, kbias, mbias, mstrides, p, nh, scale):
        H = qkv.shape[2] // 3
        q, k, v = qkv[..., :H], qkv[..., H:2 * H], qkv[..., 2 * H:]
        out, lse, ctx.seed, ctx.off = _attn_forward(q, k, v, nh, kbias, mbias, mstrides, p, scale)
        ctx.save_for_backward(qkv, kbias, mbias, out, lse)
        ctx.p, ctx.nh, ctx.scale, ctx.mstrides = p, nh, scale, mstrides
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, kbias, mbias, out, lse = ctx.saved_tensors
        H = qkv.shape[2] // 3
        dqkv = torch.empty_like(qkv)
        _attn_backward(ctx, dout, qkv[..., :H], qkv[..., H:2 * H], qkv[..., 2 * H:], out, lse, kbias, mbias,
                       dqkv[..., :H], dqkv[..., H:2 * H], dqkv[..., 2 * H:])
        return dqkv, None, None, None, None, None, None


class _Attention(torch.autograd.Function):
    """``det_attention.hip`` on separate Q [B, Lq, H] and K/V [B, Lk, H] views (cross-attention,
    DETR's projections with positional embeddings)."""

    @staticmethod
    def forward(ctx, q, k, v, kbias, mbias, mstrides, p, nh, scale):
        out, lse, ctx.seed, ctx.off = _attn_forward(q, k, v, nh, kbias, mbias, mstrides, p, scale)
        ctx.save_for_backward(q, k, v, kbias, mbias, out, lse)
        ctx.p, ctx.nh, ctx.scale, ctx.mstrides = p, nh, scale, mstrides
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, kbias, mbias, out, lse = ctx.saved_tensors
        dq = torch.empty(q.shape, dtype=q.dtype, device=q.device)
        dk = torch.empty(k.shape, dtype=k.dtype, device=k.device)
        dv = torch.empty(v.shape, dtype=v.dtype, device=v.device)
        _attn_backward(ctx, dout, q, k, v, out, lse, kbias, mbias, dq, dk, dv)
        return dq, dk, dv, None, None, None, None, None, None


# ------------------------------------------------------------------------------------------------
# public functional API (composite reference on CPU / uncovered layouts)
# ------------------------------------------------------------------------------------------------
def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None, *,
           acc: Optional[SharedWeightGrads] = None, link: Optional[ResidualGradLink] = None) -> torch.Tensor:
    """``link``: x is also a later ``linear_dropout_add_layernorm``'s residual (ResidualGradLink)."""
    (x, weight, bias), ac = _autocast(x, weight, bias)
    if not _native(x, weight, bias, width=weight.shape[0]):
        return F.linear(x, weight, bias)
    with torch.autocast("cuda", enabled=False) if ac else _null():
        return _Linear.apply(x, weight, bias, _track(acc, weight), _arm(link, x))


def linear_gelu(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None,
                approximate: str = "none", *, acc: Optional[SharedWeightGrads] = None,
                link: Optional[ResidualGradLink] = None) -> torch.Tensor:
    """``gelu(x W^T + b)``; ``approximate="tanh"`` is HF's ``gelu_new`` (ALBERT, GPT-2)."""
    (x, weight, bias), ac = _autocast(x, weight, bias)
    if not _native(x, weight, bias, width=weight.shape[0]):
        return F.gelu(F.linear(x, weight, bias), approximate=approximate)
    with torch.autocast("cuda", enabled=False) if ac else _null():
        return _LinearGELU.apply(x, weight, bias, approximate == "tanh", _track(acc, weight), _arm(link, x))


def linear_dropout_add_layernorm(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
                                 residual: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, p: float = 0.0,
                                 eps: float = 1e-12, training: bool = True, *,
                                 acc: Optional[SharedWeightGrads] = None,
                                 link: Optional[ResidualGradLink] = None) -> torch.Tensor:
    """``LayerNorm(dropout(x W^T + b) + residual)`` — BERT's SelfOutput / Output block."""
    p = float(p) if training else 0.0
    (x, weight, bias, residual, gamma, beta), ac = _autocast(x, weight, bias, residual, gamma, beta)
    if not _native(x, weight, bias, residual, gamma, beta, width=weight.shape[0], max_width=_MAX_H):
        h = F.dropout(F.linear(x, weight, bias), p, training)
        return F.layer_norm(h + residual, (weight.shape[0],), gamma, beta, eps)
    with torch.autocast("cuda", enabled=False) if ac else _null():
        return _LinearDropAddLN.apply(x, weight, bias, residual, gamma, beta, p, float(eps), _track(acc, weight), link)


def layer_norm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-12) -> torch.Tensor:
    (x, gamma, beta), ac = _autocast(x, gamma, beta)
    if not _native(x, gamma, beta, width=x.shape[-1], max_width=_MAX_H):
        return F.layer_norm(x, (x.shape[-1],), gamma, beta, eps)
    with torch.autocast("cuda", enabled=False) if ac else _null():
        return _LayerNorm.apply(x, gamma, beta, float(eps))


class _Embed(torch.autograd.Function):
    """word[ids] + type[tt] + pos[arange(S)] (det_embed.hip): a graph-safe, deterministic backward
    (torch's sorts the ids and sizes launches from a host-read count, which a hipGraph freezes)."""

    @staticmethod
    def forward(ctx, ids, tt, ww, wt, wp, pad):  # type: ignore[override]
        B, S = ids.shape
        H = ww.shape[1]
        out = torch.empty(B, S, H, dtype=ww.dtype, device=ww.device)
        ids_c = ids.contiguous().long()
        tt_c = tt.contiguous().long() if tt is not None else None
        bf = 1 if ww.dtype == torch.bfloat16 else 0
        _lib.check(_lib.get_lib().det_embed_fwd(_stream(ww), bf, ids_c.data_ptr(), tt_c.data_ptr() if tt_c is not None else None,
                                                ww.data_ptr(), wt.data_ptr(), wp.data_ptr(), out.data_ptr(), B * S, S, H),
                   "det_embed_fwd")
        ctx.save_for_backward(ids_c, tt_c if tt_c is not None else torch.zeros_like(ids_c))
        ctx.params = (ww, wt, wp)
        ctx.pad = -1 if pad is None else int(pad)
        return out

    @staticmethod
    def backward(ctx, g):  # type: ignore[override]
        ids, tt = ctx.saved_tensors
        ww, wt, wp = ctx.params
        B, S = ids.shape
        H = ww.shape[1]
        g = g.contiguous().to(ww.dtype)
        # inside a capture with the gradients pinned to the arena: accumulate in place (the rows of
        # absent ids stay as they are); otherwise fresh gradients back to autograd
        direct = torch.cuda.is_current_stream_capturing() and all(
            p.grad is not None and p.grad.is_contiguous() and p.grad.dtype == p.dtype for p in (ww, wt, wp))
        if direct:
            dww, dwt, dwp, acc = ww.grad, wt.grad, wp.grad, 1
        else:
            dww, dwt, dwp, acc = torch.zeros_like(ww), torch.empty_like(wt), torch.zeros_like(wp), 0
        lib = _lib.get_lib()
        ws = torch.empty(int(lib.det_embed_ws_floats(B * S, H, wt.shape[0])), dtype=torch.float32, device=g.device)
        _lib.check(lib.det_embed_bwd(_stream(g), 1 if ww.dtype == torch.bfloat16 else 0, ids.data_ptr(), tt.data_ptr(),
                                     g.data_ptr(), dww.data_ptr(), dwt.data_ptr(), dwp.data_ptr(), B * S, S, H, wt.shape[0],
                                     ctx.pad, ws.data_ptr(), acc), "det_embed_bwd")
        if direct:
            from determined_1_amd.ops.arena import notify_direct_grads

            notify_direct_grads((ww, wt, wp))  # autograd's post-accumulate hooks never see these
            return None, None, None, None, None, None
        return None, None, dww, dwt, dwp, None


def bert_embeddings(input_ids: torch.Tensor, token_type_ids: Optional[torch.Tensor], word: torch.Tensor,
                    token_type: torch.Tensor, position: torch.Tensor, padding_idx: Optional[int]) -> torch.Tensor:
    """word[input_ids] + token_type[token_type_ids] + position[arange(S)] -> [B, S, H] in one launch,
    with the graph-safe native backward on the GPU (torch's composition elsewhere)."""
    B, S = input_ids.shape
    native = (input_ids.is_cuda and _lib.lib_available() and word.dtype in (torch.bfloat16, torch.float32)
              and word.dtype == token_type.dtype == position.dtype and B * S <= 8192 and S <= position.shape[0]
              and word.shape[0] < (1 << 18) and token_type.shape[0] <= 4 and word.is_contiguous()
              and token_type.is_contiguous() and position.is_contiguous() and not torch.is_autocast_enabled())
    if not native:
        pos = torch.arange(S, device=input_ids.device)
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        return F.embedding(input_ids, word, padding_idx) + F.embedding(token_type_ids, token_type) + F.embedding(pos, position)
    return _Embed.apply(input_ids, token_type_ids, word, token_type, position, padding_idx)


def _composite_attention(q, k, v, nh, bias, p, scale):
    B, Lq, H = q.shape
    hd = H // nh

    def heads(t):
        return t.reshape(B, t.shape[1], nh, hd).transpose(1, 2)

    ctx = F.scaled_dot_product_attention(heads(q), heads(k), heads(v), attn_mask=bias, dropout_p=p, scale=scale)
    return ctx.transpose(1, 2).reshape(B, Lq, H)


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, num_heads: int, *,
              attn_bias: Optional[torch.Tensor] = None, p: float = 0.0, training: bool = True,
              scale: Optional[float] = None) -> torch.Tensor:
    """Multi-head attention on token-major tensors: q [B, Lq, H], k/v [B, Lk, H] (H = heads x
    head_dim; any token stride, e.g. slices of a packed projection) -> [B, Lq, H].  ``attn_bias``
    is an SDPA ``attn_mask`` (additive float or boolean keep-mask) broadcastable to
    [B, heads, Lq, Lk]; a [B, 1, 1, Lk] mask takes the per-key-row path."""
    p = float(p) if training else 0.0
    (q, k, v, attn_bias), ac = _autocast(q, k, v, attn_bias)
    B, Lq, H = q.shape
    Lk, hd = k.shape[1], H // num_heads
    scale = hd ** -0.5 if scale is None else float(scale)
    if not (q.is_cuda and q.dtype == k.dtype == v.dtype and q.dtype in _ATTN_DT
            and all(_view_ok(t, hd) for t in (q, k, v)) and v.shape[1] == Lk
            and (attn_bias is None or not attn_bias.requires_grad)
            and mfma_attention_supported(Lq, hd, q.dtype, Lk)):
        if q.is_cuda:
            FALLBACKS["count"] += 1
        return _composite_attention(q, k, v, num_heads, attn_bias, p, scale)
    kbias, mbias, mstrides = _bias_args(attn_bias, B, num_heads, Lq, Lk)
    with torch.autocast("cuda", enabled=False) if ac else _null():
        return _Attention.apply(q, k, v, kbias, mbias, mstrides, p, num_heads, scale)


def qkv_self_attention(qkv: torch.Tensor, num_heads: int, mask_bias: Optional[torch.Tensor] = None, p: float = 0.0,
                       training: bool = True) -> torch.Tensor:
    """softmax(Q K^T / sqrt(d) + mask_bias) V over the heads of a fused [B, S, 3H] QKV tensor -> [B, S, H].
    ``mask_bias`` is an SDPA mask broadcastable to [B, heads, S, S] ([B, 1, 1, S] padding masks
    take the per-key-row path)."""
    p = float(p) if training else 0.0
    (qkv, mask_bias), ac = _autocast(qkv, mask_bias)
    B, S, H3 = qkv.shape
    H = H3 // 3
    hd = H // num_heads
    if not (qkv.is_cuda and qkv.dtype in _ATTN_DT and _view_ok(qkv, hd) and (H * qkv.element_size()) % 16 == 0
            and (mask_bias is None or not mask_bias.requires_grad)
            and mfma_attention_supported(S, hd, qkv.dtype)):
        if qkv.is_cuda:
            FALLBACKS["count"] += 1
        return _composite_attention(qkv[..., :H], qkv[..., H:2 * H], qkv[..., 2 * H:], num_heads, mask_bias, p, None)
    kbias, mbias, mstrides = _bias_args(mask_bias, B, num_heads, S, S)
    with torch.autocast("cuda", enabled=False) if ac else _null():
        return _PackedQKVAttention.apply(qkv, kbias, mbias, mstrides, p, num_heads, hd ** -0.5)


def attention_dropout_mask(B: int, nh: int, S: int, p: float, seed: int, offset: int,
                           device: torch.device, Lk: Optional[int] = None) -> torch.Tensor:
    """Keep mask [B, nh, S, Lk] the MFMA attention kernels use for (p, seed, offset) (tests)."""
    Lk = S if Lk is None else Lk
    lib = _lib.get_lib()
    out = torch.empty(B, nh, S, Lk, dtype=torch.uint8, device=device)
    with torch.cuda.device(device):
        _lib.check(lib.det_attn_dropout_mask(torch.cuda.current_stream(device).cuda_stream, B, nh, S, Lk, p, seed,
                                             offset, out.data_ptr(), rng_base(device)), "det_attn_dropout_mask")
    return out.bool()


def dropout_mask(n: int, p: float, seed: int, offset: int, device: torch.device) -> torch.Tensor:
    """The keep-mask the kernels derive from (seed, offset) for n elements (tests)."""
    lib = _lib.get_lib()
    out = torch.empty(n, dtype=torch.uint8, device=device)
    with torch.cuda.device(device):
        _lib.check(lib.det_tf_dropout_mask(torch.cuda.current_stream(device).cuda_stream, n, p, seed, offset,
                                           out.data_ptr(), rng_base(device)), "det_tf_dropout_mask")
    return out.bool()


class _null:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False
