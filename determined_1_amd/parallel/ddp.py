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

RCCL knobs (the analogue of Horovod's fusion/cycle knobs, reference ``horovod.py:92-110``) come
from ``optimizations.rccl`` and are applied as NCCL_* environment before the communicator is
created (``apply_rccl_env``).
"""
import logging
import os
from typing import Any, Dict, List, MutableMapping, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from determined_1_amd.ops.arena import Arena
from determined_1_amd.ops.functional import scale_cast_, sum_rows_

MB = 1024 * 1024
MIN_BUCKET_BYTES = 2 * MB
TARGET_BUCKETS = 8
REDUCTIONS = ("fp32_accum", "allreduce")


def auto_bucket_cap(total_bytes: int, threshold_bytes: int) -> int:
    """Per-bucket byte cap: ~TARGET_BUCKETS buckets, never below 2 MB, never above the
    configured ``tensor_fusion_threshold``."""
    cap = max(MIN_BUCKET_BYTES, total_bytes // TARGET_BUCKETS)
    return int(min(threshold_bytes, cap))


class _Bucket:
    __slots__ = ("arena", "lo", "hi", "params", "comp", "recv", "work", "mode")

    def __init__(self, arena: Arena, lo: int, hi: int, params: List[int]) -> None:
        self.arena = arena
        self.lo = lo
        self.hi = hi
        self.params = params
        self.comp = None  # type: Optional[torch.Tensor]
        self.recv = None  # type: Optional[torch.Tensor]
        self.work = None  # type: Any
        self.mode = "allreduce"

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
    ) -> None:
        if reduction not in REDUCTIONS:
            raise ValueError(f"grad_reduction must be one of {REDUCTIONS}, got {reduction!r}")
        self.arenas = list(arenas)
        self.world_size = world_size
        self.rank = dist.get_rank(group) if rank is None and dist.is_initialized() else (rank or 0)
        self.group = group
        self.compression = compression
        total = sum(a.numel * a.flat_grad.element_size() for a in self.arenas)
        self.cap_bytes = auto_bucket_cap(total, int(cap_mb * MB))
        self.buckets = plan_buckets(self.arenas, self.cap_bytes)
        self._side = None  # type: Any
        for b in self.buckets:
            if compression is not None:
                b.comp = torch.empty(b.hi - b.lo, dtype=compression, device=b.arena.device)
            wire_dtype = compression if compression is not None else b.arena.flat_grad.dtype
            n = b.hi - b.lo
            if reduction == "fp32_accum" and wire_dtype in (torch.bfloat16, torch.float16) and n % world_size == 0:
                b.mode = "fp32_accum"
                b.recv = torch.empty(n, dtype=wire_dtype, device=b.arena.device)
        self._pending = [0] * len(self.buckets)
        self._ready = [False] * len(self.buckets)
        self._next = 0
        self._comm = False
        self._launched_any = False
        self._handles = []
        self._sink = None  # type: Any
        self._bucket_of = {}  # type: Dict[int, int]
        for bi, b in enumerate(self.buckets):
            for pi in b.params:
                self._bucket_of[id(b.arena.params[pi])] = bi
        for a in self.arenas:
            for p in a.params:
                self._handles.append(p.register_post_accumulate_grad_hook(self._hook))
        logging.info("gradient bucketer: %d buckets (cap %.1f MB of %.1f MB), reduction=%s, compression=%s",
                     len(self.buckets), self.cap_bytes / MB, total / MB,
                     sorted({b.mode for b in self.buckets}), compression)

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
        if self._side is not None:
            torch.cuda.current_stream(self._side.device).wait_stream(self._side)
        self._comm = False
        return True


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
