"""Bucketed, backward-overlapped gradient reduction over RCCL/xGMI on flat arenas.

Replaces ``hvd.DistributedOptimizer`` (reference ``_pytorch_context.py:152-204``; SURVEY C-1).

Design (MI355X-first, not a translation of Horovod's per-tensor async + 5 ms fusion cycle):
  * gradients already live in contiguous arenas (``ops/arena.py``) laid out in reverse
    registration order, so a bucket is a *slice* of ``flat_grad`` -- no pack/unpack copies;
  * a bucket-complete notification (GradSink flush or per-parameter hook) launches the bucket's
    collective immediately, in strict bucket order so every rank issues identical collective
    sequences (buckets that complete out of order wait for their predecessors);
  * RCCL runs on ProcessGroupNCCL's own HIP stream (event-synchronised with the compute stream),
    so the reduction of bucket k overlaps the backward of layers < k;
  * SUM is used: the 1/world_size (and 1/aggregation_frequency, AMP 1/loss_scale) factors are
    folded into the fused optimizer's single gradient read (``ops/optim.py``).

Bucket plan (``plan_buckets``): the cap is ``min(tensor_fusion_threshold, grad_bytes / 8)``
clamped to [2 MB, threshold] -- about eight buckets per model.  On an 8x MI355X node each GPU
has 7 point-to-point xGMI links; a few-MB bucket already keeps them busy far above the ~20-40 us
per-collective floor, while small buckets let communication start early in backward.  Planning
runs from the arena TAIL (the first layers, whose gradients arrive last) with a quarter-size
tail bucket, so the one collective that cannot overlap anything is short.

Reduction of 16-bit buckets (bf16 O2 arenas, or any arena with gradient compression) defaults to
``fp32_accum``: a ring all-reduce in bf16 rounds after every hop, so an 8-rank sum carries up to
7 roundings.  Instead each bucket is reduce-scattered as an **all-to-all** over the xGMI mesh
(every rank sends shard j straight to rank j -- on a fully connected node that drives all 7
links at once, no hop-by-hop arithmetic), each rank sums its N received copies in fp32 with the
``det_sum_rows`` HIP kernel (ONE rounding), and an in-place all-gather returns the reduced
bucket.  Bytes on the wire equal a ring all-reduce: 2 (N-1)/N x bucket.  ``grad_reduction:
allreduce`` selects the plain RCCL all-reduce instead.  fp32 buckets always use the RCCL
all-reduce.

``grad_reduction: auto`` measures both algorithms on every bucket size of this model at the
bucketer's construction (a few ms of collectives on scratch buffers, all ranks together), takes
the MAX over ranks of each timing with one all-reduce -- so every rank holds bit-identical
numbers and picks the identical per-bucket mode without a broadcast -- and keeps ``fp32_accum``
(one rounding) unless the RCCL all-reduce is at least ``AUTO_MARGIN`` faster.

Tensor-fusion autotune (``optimizations.auto_tune_tensor_fusion``, reference ``horovod.py:98-103``
``--autotune --autotune-log-file``): the bucket cap is searched over ``AUTOTUNE_CAPS_MB`` during
the first aggregation windows.  Each candidate runs ``AUTOTUNE_WINDOWS`` windows (the first is
discarded); a window's time is the device time from the start of its backward to the end of the
gradient synchronisation (HIP events).  The decision is taken at a fixed window index on every
rank from MAX-all-reduced timings, the buckets are re-planned (``replan``; the GradSink groups
follow through ``replan_listeners``) and every candidate is logged as CSV like Horovod's
autotune log.  ``tensor_fusion_cycle_time`` has no analogue: buckets launch the moment backward
completes them (no background cycle), so the key is accepted and ignored with an info line.

RCCL knobs (the analogue of Horovod's fusion/cycle knobs, reference ``horovod.py:92-110``) come
from ``optimizations.rccl`` and are applied as NCCL_* environment before the communicator is
created (``apply_rccl_env``).
"""
import logging
import os
import time
from typing import Any, Callable, Dict, List, MutableMapping, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from determined_1_amd.ops.arena import Arena
from determined_1_amd.ops.functional import scale_cast_, sum_rows_

MB = 1024 * 1024
MIN_BUCKET_BYTES = 2 * MB
TARGET_BUCKETS = 8
REDUCTIONS = ("fp32_accum", "allreduce", "auto")
AUTO_MARGIN = 0.10  # auto keeps fp32_accum unless the all-reduce is >= 10 % faster
AUTOTUNE_CAPS_MB = (0.5, 1, 2, 4, 8, 16, 32, 64, 128)
AUTOTUNE_WINDOWS = 3  # per candidate; the first is warmup


def auto_bucket_cap(total_bytes: int, threshold_bytes: int) -> int:
    """Per-bucket byte cap: ~TARGET_BUCKETS buckets, never below 2 MB, never above the
    configured ``tensor_fusion_threshold``."""
    cap = max(MIN_BUCKET_BYTES, total_bytes // TARGET_BUCKETS)
    return int(min(threshold_bytes, cap))


class _Bucket:
    __slots__ = ("arena", "lo", "hi", "params", "comp", "recv", "work", "mode", "f32", "f32_shard")

    def __init__(self, arena: Arena, lo: int, hi: int, params: List[int]) -> None:
        self.arena = arena
        self.lo = lo
        self.hi = hi
        self.params = params
        self.comp = None  # type: Optional[torch.Tensor]
        self.recv = None  # type: Optional[torch.Tensor]
        self.work = None  # type: Any
        self.mode = "allreduce"
        self.f32 = None  # type: Optional[torch.Tensor]  # fp32_accum under hipGraph capture (see _launch)
        self.f32_shard = None  # type: Optional[torch.Tensor]

    @property
    def grad(self) -> torch.Tensor:
        return self.arena.flat_grad[self.lo:self.hi]

    @property
    def nbytes(self) -> int:
        return (self.hi - self.lo) * self.arena.flat_grad.element_size()


def plan_buckets(arenas: Sequence[Arena], cap_bytes: int, tail_bytes: Optional[int] = None) -> List[_Bucket]:
    """Split each arena into contiguous buckets at parameter boundaries.

    Buckets are cut from the END of each arena (the earliest layers, whose gradients are produced
    last): the first cut uses ``tail_bytes`` (default cap/4), the rest ``cap_bytes``.  The list
    is returned in arena order, i.e. the order in which backward completes them."""
    if tail_bytes is None:
        tail_bytes = max(cap_bytes // 4, 1)
    out = []  # type: List[_Bucket]
    for a in arenas:
        es = a.flat_grad.element_size()
        n = len(a.params)
        cuts = []  # type: List[Tuple[int, int]]  # [first_param, last_param] inclusive, reversed
        end = n - 1
        limit = tail_bytes
        i = n - 1
        while i >= 0:
            lo = a.offsets[i]
            hi = a.offsets[end + 1] if end + 1 < n else a.numel
            if (hi - lo) * es >= limit or i == 0:
                cuts.append((i, end))
                end = i - 1
                limit = cap_bytes
            i -= 1
        for first, last in reversed(cuts):
            lo = a.offsets[first]
            hi = a.offsets[last + 1] if last + 1 < n else a.numel
            out.append(_Bucket(a, lo, hi, list(range(first, last + 1))))
    return out


def apply_rccl_env(opt: Dict[str, Any], env: Optional[MutableMapping[str, str]] = None) -> Dict[str, str]:
    """Translate ``optimizations.rccl`` into NCCL_* variables (RCCL reads them at communicator
    creation, so call before ``init_process_group``).  Explicit environment wins.

    Keys: ``algo`` (Ring/Tree), ``protocol`` (Simple/LL/LL128), ``min_channels``,
    ``max_channels``, ``buffsize`` (bytes)."""
    e = os.environ if env is None else env
    r = (opt or {}).get("rccl") or {}
    mapping = {"algo": "NCCL_ALGO", "protocol": "NCCL_PROTO", "min_channels": "NCCL_MIN_NCHANNELS",
               "max_channels": "NCCL_MAX_NCHANNELS", "buffsize": "NCCL_BUFFSIZE"}
    applied = {}
    for k, var in mapping.items():
        v = r.get(k)
        if v in (None, "", 0):
            continue
        if var not in e:
            e[var] = str(v)
            applied[var] = str(v)
    return applied


class GradientBucketer:
    def __init__(
        self,
        arenas: Sequence[Arena],
        world_size: int,
        cap_mb: float = 64.0,
        compression: Optional[torch.dtype] = None,
        group: Any = None,
        reduction: str = "fp32_accum",
        rank: Optional[int] = None,
        autotune: bool = False,
        autotune_log: Optional[str] = None,
    ) -> None:
        if reduction not in REDUCTIONS:
            raise ValueError(f"grad_reduction must be one of {REDUCTIONS}, got {reduction!r}")
        self.arenas = list(arenas)
        self.world_size = world_size
        self.rank = dist.get_rank(group) if rank is None and dist.is_initialized() else (rank or 0)
        self.group = group
        self.compression = compression
        self.reduction = reduction
        self.total_bytes = sum(a.numel * a.flat_grad.element_size() for a in self.arenas)
        self.threshold_bytes = int(cap_mb * MB)
        self.auto_choice = {}  # type: Dict[int, Dict[str, Any]]  # bucket numel -> timings + mode
        self.replan_listeners = []  # type: List[Callable[["GradientBucketer"], None]]
        self._side = None  # type: Any
        self._handles = []  # type: List[Any]
        self._sink = None  # type: Any
        self._comm = False
        self._launched_any = False
        self._plan(auto_bucket_cap(self.total_bytes, self.threshold_bytes))
        for a in self.arenas:
            for p in a.params:
                self._handles.append(p.register_post_accumulate_grad_hook(self._hook))
        self._tuner = _FusionAutotuner(self, autotune_log) if autotune else None
        # the reduction a hipGraph capture records (see _launch): forced on for the gloo CPU tests of
        # that path; launch_log, when a list, records the bucket order of every launch
        self.graph_path = False
        self.launch_log = None  # type: Optional[List[int]]

    # ------------------------------------------------------------------------------------------
    def _wire_dtype(self, b: _Bucket) -> torch.dtype:
        return self.compression if self.compression is not None else b.arena.flat_grad.dtype

    def _plan(self, cap_bytes: int) -> None:
        """(Re)build the bucket list for ``cap_bytes`` and pick each bucket's reduction."""
        self.cap_bytes = int(cap_bytes)
        self.buckets = plan_buckets(self.arenas, self.cap_bytes)
        if self.reduction == "auto":
            self._calibrate()
        downgraded = []
        for b in self.buckets:
            if self.compression is not None:
                b.comp = torch.empty(b.hi - b.lo, dtype=self.compression, device=b.arena.device)
            wire_dtype = self._wire_dtype(b)
            n = b.hi - b.lo
            want = self.reduction
            if want == "auto":
                want = self.auto_choice.get(n, {}).get("mode", "fp32_accum")
            if want == "fp32_accum" and wire_dtype in (torch.bfloat16, torch.float16):
                if n % self.world_size == 0:
                    b.mode = "fp32_accum"
                    b.recv = torch.empty(n, dtype=wire_dtype, device=b.arena.device)
                else:
                    downgraded.append(n)
        if downgraded:
            # 64-element arena alignment keeps 2/4/8 ranks exact; other world sizes can miss
            logging.warning(
                "grad_reduction fp32_accum: %d of %d buckets (numel %s) are not divisible by world size %d "
                "and fall back to a %s ring all-reduce (one rounding per hop)", len(downgraded), len(self.buckets),
                downgraded[:8], self.world_size, self._wire_dtype(self.buckets[0]))
        self.downgraded = downgraded
        self._pending = [0] * len(self.buckets)
        self._ready = [False] * len(self.buckets)
        self._next = 0
        self._bucket_of = {}  # type: Dict[int, int]
        for bi, b in enumerate(self.buckets):
            for pi in b.params:
                self._bucket_of[id(b.arena.params[pi])] = bi
        logging.info("gradient bucketer: %d buckets (cap %.1f MB of %.1f MB), reduction=%s, compression=%s",
                     len(self.buckets), self.cap_bytes / MB, self.total_bytes / MB,
                     sorted({b.mode for b in self.buckets}), self.compression)

    def replan(self, cap_bytes: int) -> None:
        """Re-cut the buckets with a new cap between aggregation windows (no collective in flight)."""
        assert not self._comm, "replan only between aggregation windows"
        self._plan(cap_bytes)
        for fn in self.replan_listeners:
            fn(self)

    def _calibrate(self, iters: int = 4) -> None:
        """``grad_reduction: auto``: time the RCCL all-reduce against all-to-all + fp32 sum +
        all-gather on each distinct bucket size (scratch buffers), MAX over ranks, pick per size."""
        sizes = sorted({b.hi - b.lo for b in self.buckets} - set(self.auto_choice))
        if not sizes:
            return
        dev = self.buckets[0].arena.device
        dt = self.compression if self.compression is not None else self.buckets[0].arena.flat_grad.dtype
        if dt not in (torch.bfloat16, torch.float16) or self.world_size == 1:
            for n in sizes:
                self.auto_choice[n] = {"mode": "fp32_accum" if dt in (torch.bfloat16, torch.float16) else "allreduce"}
            return
        times = []
        for n in sizes:
            npad = n - n % self.world_size if n % self.world_size else n
            buf = torch.randn(n, device=dev).to(dt)
            recv = torch.empty(npad, dtype=dt, device=dev)
            times.append(_time_collective(lambda: dist.all_reduce(buf, group=self.group), dev, iters))
            times.append(_time_collective(lambda: self._fp32_accum_blocking(buf[:npad], recv), dev, iters))
        t = torch.tensor(times, dtype=torch.float64, device=dev if dev.type == "cuda" else torch.device("cpu"))
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        t = t.cpu().tolist()
        for i, n in enumerate(sizes):
            ar, fa = t[2 * i], t[2 * i + 1]
            mode = "allreduce" if ar < (1.0 - AUTO_MARGIN) * fa else "fp32_accum"
            self.auto_choice[n] = {"mode": mode, "allreduce_ms": round(1e3 * ar, 4), "fp32_accum_ms": round(1e3 * fa, 4)}
        logging.info("grad_reduction auto: %s", {n: v for n, v in self.auto_choice.items() if n in sizes})

    def _fp32_accum_blocking(self, wire: torch.Tensor, recv: torch.Tensor) -> None:
        n = wire.numel() // self.world_size
        shard = wire[self.rank * n:(self.rank + 1) * n]
        dist.all_to_all_single(recv, wire, group=self.group)
        sum_rows_(recv, self.world_size, shard)
        dist.all_gather_into_tensor(wire, shard, group=self.group)

    def describe(self) -> List[Dict[str, Any]]:
        return [{"params": len(b.params), "mb": round(b.nbytes / MB, 3), "mode": b.mode} for b in self.buckets]

    def attach_sink(self, sink: Any) -> None:
        """Gradients land through ``ops.arena.GradSink`` (one batched copy per bucket): on fresh
        passes the sink announces complete buckets instead of the per-parameter hooks."""
        self._sink = sink
        sink.listeners.append(self._group_ready)

    def _group_ready(self, bi: int) -> None:
        if not self._comm:
            return
        self._ready[bi] = True
        self._launch_in_order()

    def remove(self) -> None:
        for h in self._handles:
            h.remove()
        self._handles = []

    # ------------------------------------------------------------------------------------------
    def prepare_backward(self, communicate: bool) -> None:
        """Called before every backward pass; ``communicate`` says whether this pass ends an
        aggregation window (then buckets are reduced as they complete)."""
        if communicate and self._tuner is not None:
            self._tuner.window_start()
        self._comm = communicate
        if self._comm:
            for bi, b in enumerate(self.buckets):
                self._pending[bi] = len(b.params)
                self._ready[bi] = False
            self._next = 0

    def _hook(self, p: torch.Tensor) -> None:
        if not self._comm or (self._sink is not None and self._sink.fresh):
            return
        bi = self._bucket_of.get(id(p))
        if bi is None:
            return
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._ready[bi] = True
            self._launch_in_order()

    def _launch_in_order(self) -> None:
        while self._next < len(self.buckets) and self._ready[self._next]:
            if self.launch_log is not None:
                self.launch_log.append(self._next)
            self._launch(self.buckets[self._next])
            self._next += 1

    def _side_stream(self, device: torch.device) -> Any:
        if self._side is None and device.type == "cuda":
            self._side = torch.cuda.Stream(device=device, priority=-1)
        return self._side

    def _launch(self, b: _Bucket) -> None:
        wire = b.grad
        if b.comp is not None:
            scale_cast_(wire, b.comp)
            wire = b.comp
        if b.mode == "allreduce":
            b.work = dist.all_reduce(wire, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        elif self.graph_path or (wire.is_cuda and torch.cuda.is_current_stream_capturing()):
            # inside a hipGraph capture (pytorch/_graph.py): RCCL's all-to-all does not capture on this
            # stack (the process faults; all-reduce, reduce-scatter and all-gather issued from the
            # capturing stream do --
            # scripts/dbg/rccl_capture.py, profiles/r6_rccl_capture.jsonl), so the one-rounding
            # reduction becomes an fp32 reduce-scatter of the widened bucket, the shard rounded to the
            # wire dtype once, and the same in-place all-gather
            n = wire.numel() // self.world_size
            if b.f32 is None or b.f32.numel() != wire.numel():
                b.f32 = torch.empty(wire.numel(), dtype=torch.float32, device=wire.device)
                b.f32_shard = torch.empty(n, dtype=torch.float32, device=wire.device)
            shard = wire[self.rank * n:(self.rank + 1) * n]
            b.f32.copy_(wire)
            # issued from the capturing stream itself: a collective chained through a side stream
            # faults the capture (rs_ag_side_chain / side_stream_chain in the probe)
            dist.reduce_scatter_tensor(b.f32_shard, b.f32, op=dist.ReduceOp.SUM, group=self.group,
                                       async_op=True).wait()
            shard.copy_(b.f32_shard)
            b.work = dist.all_gather_into_tensor(wire, shard, group=self.group, async_op=True)
        else:
            assert b.recv is not None
            n = wire.numel() // self.world_size
            shard = wire[self.rank * n:(self.rank + 1) * n]
            w1 = dist.all_to_all_single(b.recv, wire, group=self.group, async_op=True)
            side = self._side_stream(wire.device)
            if side is None:  # CPU / gloo: blocking semantics
                w1.wait()
                sum_rows_(b.recv, self.world_size, shard)
                b.work = dist.all_gather_into_tensor(wire, shard, group=self.group, async_op=True)
            else:
                # Reduce on a side stream that waits only for the all-to-all, so the compute
                # stream (backward of earlier layers) never stalls on communication.
                with torch.cuda.stream(side):
                    w1.wait()
                    sum_rows_(b.recv, self.world_size, shard)
                    b.work = dist.all_gather_into_tensor(wire, shard, group=self.group, async_op=True)
        self._launched_any = True

    def synchronize(self) -> bool:
        """Launch any bucket not yet launched (unused parameters), then make the current stream
        wait for every reduction.  Returns True if a communication round happened."""
        if not self._comm:
            return False
        for bi in range(len(self.buckets)):
            self._ready[bi] = True
        self._launch_in_order()
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                b.work = None
                if b.comp is not None:
                    scale_cast_(b.comp, b.grad)
        if self._side is not None and not torch.cuda.is_current_stream_capturing():
            # (a captured window keeps its collectives on the capturing stream: nothing to join)
            torch.cuda.current_stream(self._side.device).wait_stream(self._side)
        self._comm = False
        if self._tuner is not None:
            self._tuner.window_end()
        return True


def _time_collective(fn: Callable[[], None], dev: torch.device, iters: int) -> float:
    """Median seconds of ``fn`` (a blocking collective sequence) after one warmup call."""
    def sync() -> None:
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    fn()
    sync()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        sync()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


class _FusionAutotuner:
    """Bucket-cap search over the first aggregation windows (see the module docstring)."""

    def __init__(self, bucketer: GradientBucketer, log_path: Optional[str]) -> None:
        self.b = bucketer
        self.log_path = log_path
        self.caps = [int(c * MB) for c in AUTOTUNE_CAPS_MB if c * MB <= bucketer.total_bytes] or [bucketer.cap_bytes]
        self.window = 0
        self.marks = []  # type: List[Tuple[int, Any, Any]]  # (cap, start, end) per window
        self.cur = None  # type: Any
        self.done = False
        self.result = {}  # type: Dict[int, float]
        if self.caps[0] != bucketer.cap_bytes:
            bucketer.replan(self.caps[0])

    def _now(self) -> Any:
        dev = self.b.buckets[0].arena.device
        if dev.type == "cuda":
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def window_start(self) -> None:
        if self.done:
            return
        w, per = self.window, AUTOTUNE_WINDOWS
        if w > 0 and w % per == 0:
            k = w // per
            if k >= len(self.caps):
                self._decide()
                return
            self.b.replan(self.caps[k])
        self.cur = self._now()

    def window_end(self) -> None:
        if self.done or self.cur is None:
            return
        self.marks.append((self.b.cap_bytes, self.cur, self._now()))
        self.cur = None
        self.window += 1

    def _decide(self) -> None:
        """At the same window index on every rank: resolve the timings, MAX over ranks, keep the fastest."""
        per = {}  # type: Dict[int, List[float]]
        for i, (cap, t0, t1) in enumerate(self.marks):
            if i % AUTOTUNE_WINDOWS == 0:
                continue  # first window of each candidate: re-plan / warmup
            if isinstance(t0, float):
                dt = 1e3 * (t1 - t0)
            else:
                t1.synchronize()
                dt = t0.elapsed_time(t1)
            per.setdefault(cap, []).append(dt)
        caps = list(self.caps)
        mean = [sum(per.get(c, [0.0])) / max(1, len(per.get(c, []))) for c in caps]
        dev = self.b.buckets[0].arena.device
        t = torch.tensor(mean, dtype=torch.float64, device=dev if dev.type == "cuda" else torch.device("cpu"))
        if self.b.world_size > 1 and dist.is_initialized():
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.b.group)
        mean = t.cpu().tolist()
        self.result = {c / MB: m for c, m in zip(caps, mean)}
        best = caps[min(range(len(caps)), key=lambda i: mean[i])]
        logging.info("tensor fusion autotune: window ms by cap MB %s -> %g MB", self.result, best / MB)
        if self.log_path and self.b.rank == 0:
            with open(self.log_path, "w") as f:
                f.write("cap_mb,window_ms,chosen\n")
                for c, m in zip(caps, mean):
                    f.write(f"{c / MB:g},{m:.4f},{int(c == best)}\n")
        self.done = True
        if best != self.b.cap_bytes:
            self.b.replan(best)


def broadcast_arenas(arenas: Sequence[Arena], src: int = 0, group: Any = None) -> None:
    """One broadcast per arena of the (master) parameters (SURVEY C-2)."""
    for a in arenas:
        dist.broadcast(a.master, src=src, group=group)
        a.sync_params_from_master()


def broadcast_tensors_coalesced(tensors: Sequence[torch.Tensor], src: int = 0, group: Any = None) -> None:
    """Broadcast a list of tensors as one flat buffer per dtype (model buffers, optimizer state)."""
    by_dt = {}  # type: Dict[Tuple[torch.dtype, torch.device], List[torch.Tensor]]
    for t in tensors:
        by_dt.setdefault((t.dtype, t.device), []).append(t)
    for (dt, dev), ts in by_dt.items():
        flat = torch.cat([t.detach().reshape(-1) for t in ts]) if len(ts) > 1 else ts[0].detach().reshape(-1).clone()
        dist.broadcast(flat, src=src, group=group)
        off = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n
