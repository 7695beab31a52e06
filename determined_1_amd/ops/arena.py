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
import os
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch

ALIGN_ELEMS = 64  # 256 B for fp32: every param view starts on a full HBM burst
DIRECT_LANDING = True  # landing_buffer(): producers may write gradients straight into the arena


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


def landing_buffer(p: torch.Tensor) -> Optional[torch.Tensor]:
    """Where a backward kernel may write ``p``'s gradient directly: a fresh tensor aliasing the
    parameter's arena slot while its GradSink window is fresh and the gradient has not landed yet
    (else None).  The producer writes the GEMM output there (``torch.mm(..., out=buf)``) and returns
    it; AccumulateGrad adopts it and the sink hook sees the alias and skips the landing copy
    (``det_mt_copy`` of that parameter).  If autograd clones instead, the normal copy path runs."""
    slot = getattr(p, "_det_grad_slot", None)
    if slot is None or not DIRECT_LANDING:
        return None
    sink, gi, a, i = slot
    if not sink.fresh or i in sink._seen[gi] or p.grad is not None or (gi, i) in sink._landing_taken:
        return None  # a second producer of the same window gets its own buffer; autograd sums them
    sink._landing_taken.add((gi, i))
    return a.view(a.flat_grad, i)


# Conv weight gradients that land straight in the arena run on a side stream and overlap the
# input-gradient chain (DET_WGRAD_STREAM=0 turns it off).  The side stream forks from the current
# stream at each weight gradient and is joined (join_side_work) before anything reads the arena:
# GradSink flushes, end_backward and context.backward.  Operands stay referenced until the join, so
# the caching allocator cannot hand their blocks to the main stream while the side stream still
# reads them.  Eager ResNet-50 at batch 512: 12,68k -> 12,96-13,18k samples/s
# (profiles/r6_wgrad_side_stream_ab.jsonl).  A captured fork/join replayed bitwise equal but no
# faster (this runtime's graph launch runs the two branches one after the other), so captures do
# not fork.
SIDE_WGRAD = os.environ.get("DET_WGRAD_STREAM", "1") != "0"
# only weight gradients whose output gradient has at least this many elements fork (small convs of
# host-bound steps gain nothing from the overlap and pay the fork / join)
SIDE_MIN_ELEMS = int(os.environ.get("DET_WGRAD_STREAM_MIN", "0"))
_SIDE = {"streams": {}, "keep": [], "pending": None}  # type: Dict[str, Any]
SIDE_COUNTS = {"forks": 0, "joins": 0}


class side_work:
    """``with side_work(on, *operands):`` run the body on the device's side stream when ``on``."""

    def __init__(self, on: bool, *keep: torch.Tensor) -> None:
        # not under hipGraph capture: a replay runs the forked branch serialised anyway on this runtime,
        # so a captured step stays single-stream (simpler graphs, same numbers)
        self.on = bool(on) and SIDE_WGRAD and not torch.cuda.is_current_stream_capturing()
        self.keep = keep
        self._ctx = None

    def __enter__(self) -> "side_work":
        if not self.on:
            return self
        dev = self.keep[0].device
        main = torch.cuda.current_stream(dev)
        side = _SIDE["streams"].get(dev.index)
        if side is None:
            side = _SIDE["streams"][dev.index] = torch.cuda.Stream(dev)
        side.wait_stream(main)
        _SIDE["keep"].extend(self.keep)
        _SIDE["pending"] = (main, side)
        SIDE_COUNTS["forks"] += 1
        self._ctx = torch.cuda.stream(side)
        self._ctx.__enter__()
        return self

    def __exit__(self, *exc) -> None:
        if self._ctx is not None:
            self._ctx.__exit__(*exc)
            self._ctx = None


def join_side_work() -> None:
    """Make the stream that forked the side work wait for it, then drop the operand references."""
    pend = _SIDE["pending"]
    if pend is None:
        return
    main, side = pend
    main.wait_stream(side)
    _SIDE["pending"] = None
    _SIDE["keep"] = []
    SIDE_COUNTS["joins"] += 1


def notify_direct_grads(params: Sequence[torch.Tensor]) -> None:
    """A backward that accumulated into ``p.grad`` in place (inside a hipGraph capture, the arena
    views pinned) returns None to autograd, so AccumulateGrad -- and with it every post-accumulate
    hook -- never runs for ``p``.  Run those hooks here, in the order autograd would have, so the
    DP gradient bucketer still counts the parameter (its bucket, and the buckets behind it, launch
    on time instead of at synchronize()) and user hooks see the gradient.  Direct writers:
    transformer._Embed, cnn._CifarCNN."""
    for p in params:
        hooks = getattr(p, "_post_accumulate_grad_hooks", None)
        if hooks:
            for h in list(hooks.values()):
                h(p)


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


# (debugging) DET_SINK_CAPTURE_FOREACH=0: captured landings copy one tensor per launch
CAPTURE_FOREACH = os.environ.get("DET_SINK_CAPTURE_FOREACH", "1") != "0"


class GradSink:
    """Steal-then-batch-copy gradient landing for arena parameters.

    With ``.grad`` pinned to arena views, autograd's AccumulateGrad does one read-modify-write
    ``grad += new`` launch per parameter every step (161 launches / ~2 ms per ResNet-50 step in
    profiles/r1_resnet50_bs256_o2_fusedbn_kernel_stats.csv).  Instead, ``zero_grad`` sets
    ``.grad = None`` (marking the window *fresh*), AccumulateGrad then *steals* the freshly
    produced gradient (no kernel), and a post-accumulate hook collects it.  When every parameter
    of a group (= an all-reduce bucket, or a whole arena on one GPU) has arrived, ONE
    ``det_mt_copy`` launch moves the group's gradients into the contiguous arena slice, and the
    group's listeners (the RCCL bucketer) are notified.  Later backward passes of the same
    aggregation window accumulate in place into the arena views as before.
    """

    def __init__(self, groups: Sequence[Tuple["Arena", List[int]]]) -> None:
        self.groups = [(a, list(idx)) for a, idx in groups]
        self.group_of = {}  # type: Dict[int, int]
        for gi, (a, idx) in enumerate(self.groups):
            for i in idx:
                self.group_of[id(a.params[i])] = gi
        self.fresh = False
        self.listeners = []  # type: List[Callable[[int], None]]
        self._pending = [len(idx) for _, idx in self.groups]
        self._seen = [set() for _ in self.groups]  # type: List[set]
        self._stolen = [[] for _ in self.groups]  # type: List[List[Tuple[int, torch.Tensor]]]
        self._keep = []  # type: List[torch.Tensor]
        self._landing_taken = set()  # type: set  # (group, index) slots handed out by landing_buffer
        self._tables = {}  # type: Dict[int, Any]
        self.captured_flushes = 0  # landing copies recorded into hipGraphs (foreach copies)
        self._handles = []
        # per parameter, everything the hook compares against (one dict lookup instead of ~10
        # tensor attribute reads per parameter per backward: the hook runs 150-160 times a step)
        self._slot = {}  # type: Dict[int, Tuple[int, Arena, int, torch.Tensor, int, Any, Any, Any, Any]]
        for gi, (a, idx) in enumerate(self.groups):
            for i in idx:
                v = a.grad_views[i]
                self._slot[id(a.params[i])] = (gi, a, i, v, v.data_ptr(), v.shape, v.stride(), v.dtype, v.device)
                self._handles.append(a.params[i].register_post_accumulate_grad_hook(self._hook))
                a.params[i]._det_grad_slot = (self, gi, a, i)  # see landing_buffer()

    @staticmethod
    def for_arenas(arenas: Sequence["Arena"]) -> "GradSink":
        return GradSink([(a, list(range(len(a.params)))) for a in arenas])

    def remove(self) -> None:
        for h in self._handles:
            h.remove()
        self._handles = []

    def detach(self) -> None:
        """Stop landing gradients (hooks, direct-landing slots) and re-pin ``.grad`` to the arena
        views, leaving plain in-place accumulation.  Used before hipGraph capture: the sink's
        pointer tables are uploaded from host staging buffers that a replay must not re-read."""
        self.remove()
        for a, idx in self.groups:
            for i in idx:
                p = a.params[i]
                if getattr(p, "_det_grad_slot", None) is not None and p._det_grad_slot[0] is self:
                    del p._det_grad_slot
        self.fresh = False
        for a, _ in self.groups:
            a.zero_grad()

    def host_state(self) -> bool:
        """The window state a hipGraph replay must leave behind (pytorch/_graph.py): True = fresh
        (gradients None, the next backward steals them), False = continuing (``.grad`` pinned to the
        arena views, the next backward accumulates in place)."""
        return self.fresh

    def set_host_state(self, fresh: bool) -> None:
        """After a replay (which runs no Python): put the host side where the captured step left it."""
        if fresh:
            self.start_window()
            return
        self.fresh = False
        for a, idx in self.groups:
            for i in idx:
                a.params[i].grad = a.grad_views[i]
        self._keep = []
        self._landing_taken = set()

    def start_window(self) -> None:
        """Called by zero_grad: grads become None and the next backward steals them."""
        self.fresh = True
        for gi, (a, idx) in enumerate(self.groups):
            self._pending[gi] = len(idx)
            self._seen[gi] = set()
            self._stolen[gi] = []
            for i in idx:
                a.params[i].grad = None
        self._keep = []
        self._landing_taken = set()

    def _hook(self, p: torch.Tensor) -> None:
        if not self.fresh:
            return
        slot = self._slot.get(id(p))
        if slot is None:
            return
        gi, a, i, view, vptr, vshape, vstride, vdtype, vdev = slot
        seen = self._seen[gi]
        if i in seen:
            return
        seen.add(i)
        g = p.grad
        if g is None:
            p.grad = view
        elif g is not view:
            same = g.dtype == vdtype and g.shape == vshape and g.stride() == vstride
            if same and g.data_ptr() == vptr:
                pass  # produced in place by its backward (landing_buffer): nothing to move
            elif same and g.device == vdev:
                # same shape + the arena view's (dense) strides => g is dense with the same element order
                self._stolen[gi].append((i, g))
            else:
                with torch.no_grad():
                    view.copy_(g)
            p.grad = view
        self._pending[gi] -= 1
        if self._pending[gi] == 0:
            self._flush(gi)

    def _flush(self, gi: int) -> None:
        join_side_work()  # side-stream weight gradients landed in this group's slots
        a, idx = self.groups[gi]
        stolen = self._stolen[gi]
        self._stolen[gi] = []
        if stolen:
            if a.flat_grad.device.type == "cuda" and torch.cuda.is_current_stream_capturing() and not CAPTURE_FOREACH:
                with torch.no_grad():
                    for i, g in stolen:
                        a.grad_views[i].copy_(g)
                self.captured_flushes += 1
            elif a.flat_grad.device.type == "cuda" and torch.cuda.is_current_stream_capturing():
                # under hipGraph capture: a multi-tensor copy whose pointers travel as kernel
                # arguments.  A device pointer table allocated in the capture gets an address the
                # graph's private pool already gave a tensor freed earlier in the same step, so a
                # replay's forward overwrites it before the copy reads it (r5s22: the table written
                # once after capture faulted the first replay)
                with torch.no_grad():
                    torch._foreach_copy_([a.grad_views[i] for i, _ in stolen], [g for _, g in stolen])
                self.captured_flushes += 1
            elif a.flat_grad.device.type == "cuda":
                from determined_1_amd.ops import _lib
                from determined_1_amd.ops.functional import dtype_code

                rows = []
                max_n = 0
                for i, g in stolen:
                    n = a.numels[i]
                    rows += [g.data_ptr(), a.grad_views[i].data_ptr(), n]
                    max_n = max(max_n, n)
                dev_table = self._table(gi, rows, a.flat_grad.device)
                code = dtype_code(a.dtype)
                _lib.check(_lib.get_lib().det_mt_copy(
                    torch.cuda.current_stream(a.flat_grad.device).cuda_stream, dev_table.data_ptr(), len(stolen),
                    code, code, max_n, 1.0), "mt_copy(grad sink)")
            else:
                with torch.no_grad():
                    for i, g in stolen:
                        a.grad_views[i].copy_(g)
            self._keep.extend(g for _, g in stolen)
        for fn in self.listeners:
            fn(gi)

    def _table(self, gi: int, rows: List[int], device: torch.device) -> torch.Tensor:
        """Upload the pointer table through a double-buffered pinned staging area."""
        slot = self._tables.get(gi)
        n = len(rows)
        if slot is None or slot["cap"] < n:
            cap = max(n, 3 * 64)
            slot = {"cap": cap, "i": 0,
                    "host": [torch.empty(cap, dtype=torch.int64).pin_memory() for _ in range(2)],
                    "dev": [torch.empty(cap, dtype=torch.int64, device=device) for _ in range(2)],
                    "ev": [None, None]}
            self._tables[gi] = slot
        k = slot["i"]
        slot["i"] ^= 1
        if slot["ev"][k] is not None:
            slot["ev"][k].synchronize()  # the H2D copy that last used this staging buffer is done
        slot["host"][k][:n].copy_(torch.tensor(rows, dtype=torch.int64))
        slot["dev"][k][:n].copy_(slot["host"][k][:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        slot["ev"][k] = ev
        return slot["dev"][k]

    def end_backward(self) -> None:
        """After the first backward of a window: land stragglers (parameters that received no
        gradient get zeros) and switch to in-place accumulation for the rest of the window."""
        join_side_work()
        if not self.fresh:
            return
        for gi, (a, idx) in enumerate(self.groups):
            if self._pending[gi] <= 0:
                continue
            with torch.no_grad():
                for i in idx:
                    if i not in self._seen[gi]:
                        a.grad_views[i].zero_()
                        a.params[i].grad = a.grad_views[i]
            self._pending[gi] = 0
            self._flush(gi)
        self.fresh = False
