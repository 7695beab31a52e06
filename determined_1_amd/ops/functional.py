"""Python entry points for the gfx950 kernels, with pure-PyTorch references for CPU tensors.

Every function dispatches on the tensor's device:
  * ``cuda`` (HIP) tensors -> ``libdetkernels.so`` on the current stream (never eager fallback),
  * ``cpu`` tensors        -> a straightforward fp32 PyTorch implementation of the same math
                              (these are also the numerics references the GPU tests compare to).
"""
from typing import List, Optional, Sequence

import torch

from determined_1_amd.ops import _lib

_DT = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16, torch.float16: _lib.F16}


def dtype_code(dt: torch.dtype) -> int:
    try:
        return _DT[dt]
    except KeyError:
        raise TypeError(f"unsupported dtype for det kernels: {dt}")


def _stream_ptr(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def is_gpu(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


# ----------------------------------------------------------------------------------------------
# scale / cast
# ----------------------------------------------------------------------------------------------
def sum_rows_(src: torch.Tensor, rows: int, dst: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    """dst[:] = scale * src.view(rows, -1).sum(0) with fp32 accumulation and one final rounding
    (the shard reduction of the fp32-accumulating gradient reduce-scatter, ``parallel/ddp.py``)."""
    n = dst.numel()
    assert src.numel() == rows * n, (src.shape, rows, dst.shape)
    assert src.is_contiguous() and dst.is_contiguous()
    if is_gpu(src):
        _lib.check(
            _lib.get_lib().det_sum_rows(_stream_ptr(src), src.data_ptr(), dtype_code(src.dtype), dst.data_ptr(),
                                        dtype_code(dst.dtype), int(rows), n, float(scale)),
            "sum_rows",
        )
    else:
        s = src.view(rows, n).float().sum(0)
        if scale != 1.0:
            s = s * scale
        dst.copy_(s.view_as(dst))
    return dst


def scale_cast_(
    src: torch.Tensor,
    dst: torch.Tensor,
    scale: float = 1.0,
    scale_dev: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    """dst[:] = (src * scale * scale_dev).to(dst.dtype).  Both must be contiguous, same numel."""
    assert src.numel() == dst.numel(), (src.shape, dst.shape)
    assert src.is_contiguous() and dst.is_contiguous()
    if is_gpu(src):
        _lib.check(
            _lib.get_lib().det_scale_cast(
                _stream_ptr(src),
                src.data_ptr(),
                dtype_code(src.dtype),
                dst.data_ptr(),
                dtype_code(dst.dtype),
                src.numel(),
                float(scale),
                _ptr(scale_dev),
            ),
            "scale_cast",
        )
    else:
        s = src.float() * scale
        if scale_dev is not None:
            s = s * scale_dev.float()
        dst.copy_(s.view_as(dst))
    return dst


# ----------------------------------------------------------------------------------------------
# grad norm / non-finite detection
# ----------------------------------------------------------------------------------------------
class NormWorkspace:
    """Device scratch for multi-segment norm reductions (partials + norm + flag + clip coef).

    Allocated once per arena set so the reduction needs no allocation per step (capturable).
    """

    def __init__(self, segments: Sequence[torch.Tensor]) -> None:
        self.segments = list(segments)
        dev = self.segments[0].device
        self.offsets = []  # type: List[int]
        total = 0
        for s in self.segments:
            self.offsets.append(total)
            total += self._nparts(s)
        self.partials = torch.zeros(max(total, 1), dtype=torch.float32, device=dev)
        self.norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self.clip_coef = torch.ones(1, dtype=torch.float32, device=dev)
        self.found_inf = torch.zeros(1, dtype=torch.int32, device=dev)

    @staticmethod
    def _nparts(s: torch.Tensor) -> int:
        if is_gpu(s):
            return int(_lib.get_lib().det_sumsq_num_partials(s.numel()))
        return 1


def global_norm_(
    ws: NormWorkspace, pre_scale: float = 1.0, max_norm: float = 0.0
) -> torch.Tensor:
    """Global L2 norm of all segments (times ``pre_scale``) into ``ws.norm``; sets ``ws.found_inf``
    when non-finite and ``ws.clip_coef = min(1, max_norm/(norm+1e-6))`` when ``max_norm > 0``.

    Two launches per segment set regardless of tensor count: per-block partial sums of squares
    (one launch per contiguous segment), then a single-block finalize.
    """
    seg0 = ws.segments[0]
    if is_gpu(seg0):
        lib = _lib.get_lib()
        st = _stream_ptr(seg0)
        base = ws.partials.data_ptr()
        for s, off in zip(ws.segments, ws.offsets):
            _lib.check(
                lib.det_sumsq_partials(st, s.data_ptr(), dtype_code(s.dtype), s.numel(), base + 4 * off),
                "sumsq_partials",
            )
        _lib.check(
            lib.det_norm_finalize(
                st,
                base,
                ws.partials.numel(),
                float(pre_scale),
                float(max_norm),
                ws.norm.data_ptr(),
                ws.found_inf.data_ptr(),
                ws.clip_coef.data_ptr(),
            ),
            "norm_finalize",
        )
    else:
        sq = torch.zeros((), dtype=torch.float64)
        for s in ws.segments:
            sq = sq + (s.double() ** 2).sum()
        norm = (sq.sqrt() * pre_scale).float()
        ws.norm.fill_(norm.item())
        bad = not torch.isfinite(norm).item()
        if bad:
            ws.found_inf.fill_(1)
        c = 1.0
        if max_norm > 0 and not bad:
            c = min(1.0, max_norm / (norm.item() + 1e-6))
        ws.clip_coef.fill_(c)
    return ws.norm


def unscale_check_(x: torch.Tensor, scale: float, found_inf: torch.Tensor) -> None:
    """x *= scale in place; found_inf[0] = 1 if any result is non-finite."""
    assert x.is_contiguous()
    if is_gpu(x):
        _lib.check(
            _lib.get_lib().det_unscale_check(
                _stream_ptr(x), x.data_ptr(), dtype_code(x.dtype), x.numel(), float(scale), found_inf.data_ptr()
            ),
            "unscale_check",
        )
    else:
        x.mul_(scale)
        if not torch.isfinite(x).all():
            found_inf.fill_(1)


# ----------------------------------------------------------------------------------------------
# multi-tensor copy (coalescing buffers for broadcast; non-arena tensors)
# ----------------------------------------------------------------------------------------------
class MultiTensorCopy:
    """Copy a list of tensors into/out of one flat buffer with one launch (pointer table on device).

    ``pack()``: flat[off_i : off_i+n_i] = tensors[i] * scale  (cast to flat dtype)
    ``unpack()``: tensors[i] = flat[...] * scale               (cast to tensor dtype)
    All tensors must share one dtype and be contiguous.
    """

    def __init__(self, tensors: Sequence[torch.Tensor], flat: Optional[torch.Tensor] = None,
                 flat_dtype: Optional[torch.dtype] = None) -> None:
        self.tensors = list(tensors)
        assert self.tensors, "empty tensor list"
        dt = self.tensors[0].dtype
        assert all(t.dtype == dt and t.is_contiguous() for t in self.tensors)
        dev = self.tensors[0].device
        total = sum(t.numel() for t in self.tensors)
        if flat is None:
            flat = torch.empty(total, dtype=flat_dtype or dt, device=dev)
        assert flat.numel() == total
        self.flat = flat
        self.offsets = []
        off = 0
        for t in self.tensors:
            self.offsets.append(off)
            off += t.numel()
        self.max_numel = max(t.numel() for t in self.tensors)
        if is_gpu(flat):
            es = flat.element_size()
            rows_pack, rows_unpack = [], []
            for t, o in zip(self.tensors, self.offsets):
                rows_pack += [t.data_ptr(), flat.data_ptr() + es * o, t.numel()]
                rows_unpack += [flat.data_ptr() + es * o, t.data_ptr(), t.numel()]
            self._table_pack = torch.tensor(rows_pack, dtype=torch.int64).to(dev)
            self._table_unpack = torch.tensor(rows_unpack, dtype=torch.int64).to(dev)

    def pack(self, scale: float = 1.0) -> torch.Tensor:
        if is_gpu(self.flat):
            _lib.check(
                _lib.get_lib().det_mt_copy(
                    _stream_ptr(self.flat), self._table_pack.data_ptr(), len(self.tensors),
                    dtype_code(self.tensors[0].dtype), dtype_code(self.flat.dtype), self.max_numel, float(scale),
                ),
                "mt_copy(pack)",
            )
        else:
            for t, o in zip(self.tensors, self.offsets):
                self.flat[o:o + t.numel()].copy_(t.reshape(-1).float() * scale)
        return self.flat

    def unpack(self, scale: float = 1.0) -> None:
        if is_gpu(self.flat):
            _lib.check(
                _lib.get_lib().det_mt_copy(
                    _stream_ptr(self.flat), self._table_unpack.data_ptr(), len(self.tensors),
                    dtype_code(self.flat.dtype), dtype_code(self.tensors[0].dtype), self.max_numel, float(scale),
                ),
                "mt_copy(unpack)",
            )
        else:
            for t, o in zip(self.tensors, self.offsets):
                t.copy_((self.flat[o:o + t.numel()].float() * scale).view_as(t))


# ----------------------------------------------------------------------------------------------
# input pipeline
# ----------------------------------------------------------------------------------------------
def u8_normalize(
    images_u8_nhwc: torch.Tensor,
    mean: Sequence[float],
    std: Sequence[float],
    out_dtype: torch.dtype = torch.bfloat16,
    pad4: bool = False,
) -> torch.Tensor:
    """uint8 NHWC [N,H,W,C] -> normalized float tensor of logical shape [N,C,H,W] in
    channels_last memory format (no transpose pass: NHWC bytes are already channels_last).
    ``pad4`` (bf16, C <= 3): emit 4 channels, the last one zero -- the input layout of the native
    ResNet stem (``ops.conv.stem_conv``)."""
    x = images_u8_nhwc
    assert x.dtype == torch.uint8 and x.dim() == 4 and x.is_contiguous()
    n, h, w, c = x.shape
    pad4 = pad4 and c <= 3 and out_dtype == torch.bfloat16
    co = 4 if pad4 else c
    out = torch.empty((n, co, h, w), dtype=out_dtype, device=x.device, memory_format=torch.channels_last)
    if is_gpu(x):
        import ctypes

        m = (ctypes.c_float * 4)(*[float(v) for v in mean] + [0.0] * (4 - len(mean)))
        s = (ctypes.c_float * 4)(*[float(v) for v in std] + [1.0] * (4 - len(std)))
        fn = _lib.get_lib().det_u8_normalize_pad4 if pad4 else _lib.get_lib().det_u8_normalize
        _lib.check(
            fn(
                _stream_ptr(x), x.data_ptr(), out.data_ptr(), dtype_code(out_dtype), n * h * w if pad4 else x.numel(), c,
                ctypes.cast(m, ctypes.c_void_p), ctypes.cast(s, ctypes.c_void_p),
            ),
            "u8_normalize",
        )
    else:
        mt = torch.tensor(mean, dtype=torch.float32)
        st = torch.tensor(std, dtype=torch.float32)
        y = (x.float() - mt) / st  # NHWC
        if pad4:
            out.zero_()
        out[:, :c].copy_(y.permute(0, 3, 1, 2))
    return out
