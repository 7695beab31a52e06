"""Flat parameter / gradient arenas.

MI355X-first replacement for Horovod tensor fusion (reference:
``harness/determined/pytorch/_pytorch_context.py:152-204`` wraps the optimizer in
``hvd.DistributedOptimizer`` which packs per-parameter gradients into <=64 MB fusion buffers every
cycle and unpacks them afterwards).

Here every parameter of an optimizer param group is *re-homed* into one contiguous buffer
(``flat_param``) and its ``.grad`` is pinned to a view of a matching ``flat_grad``:

  * autograd accumulates straight into the arena (AccumulateGrad adds in place into an existing
    ``.grad``), so there is no pack/unpack pass at all;
  * a gradient all-reduce bucket is a contiguous slice of ``flat_grad`` (see
    ``determined_1_amd/parallel/ddp.py``) -- large, few collectives over xGMI;
  * the fused optimizer (``optim.py``) is one HIP launch per arena;
  * for bf16/fp16 params an fp32 ``master`` copy is kept (apex O2 master weights), and the
    optimizer kernel writes the updated low-precision copy back in the same pass.

Parameters are laid out in REVERSE registration order: backward produces gradients roughly from
the last layer to the first, so buckets become ready front-to-back along the arena.
"""
from typing import Dict, List, Optional, Sequence

import torch

ALIGN_ELEMS = 64  # 256 B for fp32: every param view starts on a full HBM burst


def _round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


def _dense_strides(p: torch.Tensor) -> Sequence[int]:
    """Strides to use for the arena view of ``p``: keep channels_last if the param has it."""
    if p.dim() == 4 and not p.is_contiguous() and p.is_contiguous(memory_format=torch.channels_last):
        return p.stride()
    if p.dim() == 5 and not p.is_contiguous() and p.is_contiguous(memory_format=torch.channels_last_3d):
        return p.stride()
    return torch.empty(p.shape, device="meta").stride()


class Arena:
    """One flat storage holding a list of same-dtype parameters, their grads and fp32 master."""

    def __init__(self, params: List[torch.nn.Parameter], device: torch.device, reverse: bool = True) -> None:
        assert params, "empty arena"
        dt = params[0].dtype
        assert all(p.dtype == dt for p in params)
        assert dt in (torch.float32, torch.bfloat16, torch.float16), dt
        self.params = list(reversed(params)) if reverse else list(params)
        self.dtype = dt
        self.device = device
        self.offsets = []  # type: List[int]
        self.numels = []  # type: List[int]
        self.strides = []  # type: List[Sequence[int]]
        off = 0
        for p in self.params:
            self.offsets.append(off)
            self.numels.append(p.numel())
            self.strides.append(_dense_strides(p))
            off = _round_up(off + p.numel(), ALIGN_ELEMS)
        self.numel = max(off, ALIGN_ELEMS)
        self.flat_param = torch.zeros(self.numel, dtype=dt, device=device)
        self.flat_grad = torch.zeros(self.numel, dtype=dt, device=device)
        self.param_views = []  # type: List[torch.Tensor]
        self.grad_views = []  # type: List[torch.Tensor]
        with torch.no_grad():
            for i, p in enumerate(self.params):
                v = self.view(self.flat_param, i)
                v.copy_(p.data)
                self.param_views.append(v)
                p.data = v
                gv = self.view(self.flat_grad, i)
                if p.grad is not None:
                    gv.copy_(p.grad)
                self.grad_views.append(gv)
                p.grad = gv
        if dt == torch.float32:
            self.master = self.flat_param
        else:
            self.master = self.flat_param.float()
        self.index = {id(p): i for i, p in enumerate(self.params)}  # type: Dict[int, int]

    @property
    def has_master(self) -> bool:
        return self.master is not self.flat_param

    def view(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        p = self.params[i]
        return torch.as_strided(flat, p.shape, self.strides[i], self.offsets[i])

    def ensure_grads(self) -> None:
        """Re-pin ``.grad`` to the arena if user code replaced or dropped it."""
        for p, gv in zip(self.params, self.grad_views):
            g = p.grad
            if g is gv:
                continue
            with torch.no_grad():
                if g is None:
                    gv.zero_()
                else:
                    gv.copy_(g)
            p.grad = gv

    def zero_grad(self) -> None:
        self.flat_grad.zero_()
        # A user may have set .grad = None through torch APIs; re-pin without copying.
        for p, gv in zip(self.params, self.grad_views):
            if p.grad is not gv:
                p.grad = gv

    @torch.no_grad()
    def sync_master_from_params(self) -> None:
        if self.has_master:
            self.master.copy_(self.flat_param)

    @torch.no_grad()
    def sync_params_from_master(self) -> None:
        if self.has_master:
            self.flat_param.copy_(self.master)

    def param_slice_for(self, start_param: int, end_param: int) -> slice:
        """Element range covering params [start_param, end_param) (arena order)."""
        lo = self.offsets[start_param]
        hi = self.offsets[end_param] if end_param < len(self.params) else self.numel
        return slice(lo, hi)


def build_arenas(params: Sequence[torch.nn.Parameter], device: torch.device) -> List[Arena]:
    """Group ``params`` (one optimizer param group) by dtype and build one arena per dtype.

    Parameters that cannot live in an arena (sparse, non-float, not requiring grad, or already
    in another arena) are rejected with ValueError so the caller can fall back explicitly.
    """
    by_dtype = {}  # type: Dict[torch.dtype, List[torch.nn.Parameter]]
    for p in params:
        if not p.requires_grad:
            continue
        if p.is_sparse or p.dtype not in (torch.float32, torch.bfloat16, torch.float16):
            raise ValueError(f"parameter of dtype {p.dtype} / layout {p.layout} cannot be arena-allocated")
        if p.device != device:
            raise ValueError(f"parameter on {p.device}, arena device is {device}")
        by_dtype.setdefault(p.dtype, []).append(p)
    return [Arena(ps, device) for ps in by_dtype.values()]


def arenas_grad_segments(arenas: Sequence[Arena]) -> List[torch.Tensor]:
    return [a.flat_grad for a in arenas]


def find_arena(arenas: Sequence[Arena], p: torch.Tensor) -> Optional[Arena]:
    for a in arenas:
        if id(p) in a.index:
            return a
    return None
