"""Bucketed, backward-overlapped gradient all-reduce over RCCL/xGMI on flat arenas.

Replaces ``hvd.DistributedOptimizer`` (reference ``_pytorch_context.py:152-204``; SURVEY C-1).

Design (MI355X-first, not a translation of Horovod's per-tensor async + 5 ms fusion cycle):
  * gradients already live in contiguous arenas (``ops/arena.py``) laid out in reverse
    registration order, so a bucket is a *slice* of ``flat_grad`` -- no pack/unpack copies;
  * a ``post_accumulate_grad`` hook per parameter counts down its bucket; when a bucket is
    complete it is all-reduced immediately (``async_op=True``), in strict bucket order so every
    rank issues identical collective sequences (buckets that complete out of order wait for their
    predecessors);
  * RCCL runs on its own HIP stream (ProcessGroupNCCL's internal stream, event-synchronised with
    the compute stream), so the all-reduce of bucket k overlaps the backward of layers < k;
  * SUM (not AVG) is used: the 1/world_size (and 1/aggregation_frequency, AMP 1/loss_scale)
    factors are folded into the fused optimizer's single gradient read (``ops/optim.py``);
  * optional compression casts each bucket to bf16 (MI355X-native; fp16 also accepted) with the
    ``det_scale_cast`` kernel before the collective and back after it;
  * bucket size comes from ``optimizations.tensor_fusion_threshold`` (MB, default 64, as the
    reference).  On an 8x MI355X node each GPU has 7 xGMI links (~153 GB/s each); a 64 MB ring
    all-reduce moves ~2*(7/8)*64 MB per GPU which keeps every link busy for ~0.1 ms+, well above
    the per-collective launch/latency floor, while the smaller first bucket starts communication
    early in backward.
"""
import logging
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from determined_1_amd.ops.arena import Arena
from determined_1_amd.ops.functional import scale_cast_

FIRST_BUCKET_BYTES = 4 * 1024 * 1024


class _Bucket:
    __slots__ = ("arena", "lo", "hi", "params", "comp", "work")

    def __init__(self, arena: Arena, lo: int, hi: int, params: List[int]) -> None:
        self.arena = arena
        self.lo = lo
        self.hi = hi
        self.params = params
        self.comp = None  # type: Optional[torch.Tensor]
        self.work = None  # type: Any

    @property
    def grad(self) -> torch.Tensor:
        return self.arena.flat_grad[self.lo:self.hi]


def plan_buckets(arenas: Sequence[Arena], cap_bytes: int, first_bytes: int = FIRST_BUCKET_BYTES) -> List[_Bucket]:
    """Split each arena into contiguous buckets at parameter boundaries."""
    buckets = []  # type: List[_Bucket]
    for a in arenas:
        es = a.flat_grad.element_size()
        start = 0
        cur = []  # type: List[int]
        limit = min(first_bytes, cap_bytes) if not buckets else cap_bytes
        for i in range(len(a.params)):
            cur.append(i)
            lo = a.offsets[start]
            hi = a.offsets[i + 1] if i + 1 < len(a.params) else a.numel
            if (hi - lo) * es >= limit:
                buckets.append(_Bucket(a, lo, hi, cur))
                cur = []
                start = i + 1
                limit = cap_bytes
        if cur:
            lo = a.offsets[start]
            buckets.append(_Bucket(a, lo, a.numel, cur))
    return buckets


class GradientBucketer:
    def __init__(
        self,
        arenas: Sequence[Arena],
        world_size: int,
        cap_mb: float = 64.0,
        compression: Optional[torch.dtype] = None,
        group: Any = None,
    ) -> None:
        self.arenas = list(arenas)
        self.world_size = world_size
        self.group = group
        self.compression = compression
        self.buckets = plan_buckets(self.arenas, int(cap_mb * 1024 * 1024))
        self._bucket_of = {}  # type: Dict[int, int]
        for bi, b in enumerate(self.buckets):
            for pi in b.params:
                self._bucket_of[id(b.arena.params[pi])] = bi
            if compression is not None:
                b.comp = torch.empty(b.hi - b.lo, dtype=compression, device=b.arena.device)
        self._pending = [0] * len(self.buckets)
        self._ready = [False] * len(self.buckets)
        self._next = 0
        self._comm = False
        self._launched_any = False
        self._handles = []
        self._sink = None  # type: Any
        for a in self.arenas:
            for p in a.params:
                self._handles.append(p.register_post_accumulate_grad_hook(self._hook))
        logging.debug("gradient bucketer: %d buckets (%s MB cap), compression=%s", len(self.buckets), cap_mb,
                      compression)

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
        aggregation window (then buckets all-reduce as they complete)."""
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

    def _launch(self, b: _Bucket) -> None:
        buf = b.grad
        if b.comp is not None:
            scale_cast_(buf, b.comp)
            buf = b.comp
        b.work = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._launched_any = True

    def synchronize(self) -> bool:
        """Launch any bucket not yet launched (unused parameters), then make the current stream
        wait for every all-reduce.  Returns True if a communication round happened."""
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
