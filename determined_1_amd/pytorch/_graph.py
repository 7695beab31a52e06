"""HIP-graph replay of ``train_batch`` (``optimizations.hip_graph: true``).

Small models (the CIFAR-10 CNN of the ASHA benchmark) are launch-bound on an MI355X: a batch of
forward + backward + fused optimizer step is ~60 kernels of a few microseconds each, while the
Python/dispatcher cost of issuing them is ~1.5 ms (``scripts/bench_cifar_trial.py``), so the GPU
idles ~90% of a trial (``profiles/r2_asha_baseline_shape.json``).  The reference has no
counterpart (it runs eager PyTorch under Horovod); the MI355X-first answer is to capture the whole
user ``train_batch`` -- autograd, the arena optimizer's fused HIP kernel, ``zero_grad`` -- into one
hipGraph and replay it per batch: one launch, no per-kernel host work.

Why it is safe here: the arena design already keeps every tensor a step touches at a fixed
address (flat parameter/gradient/optimizer-state arenas), so a replay sees the same memory as the
capture.  What is NOT in the graph and is handled on the host:

  * inputs: each batch is copied into the static input tensors the graph was captured with;
  * outputs: the returned metric tensors are static; they are cloned before the next replay;
  * optimizer bookkeeping: ``FusedOptimizer.graph_replayed()`` advances step counters;
  * anything that changes kernel arguments (input shapes, learning rate / other
    hyper-parameters, SGD's first-step flag, the epoch index passed to ``train_batch``) is part
    of the graph key: a new key runs eagerly for ``WARMUP`` batches (lazy state, MIOpen find),
    then is captured.  A key that keeps changing (per-batch LR schedules) turns graphs off.

Requirements on user code (documented in the README): ``train_batch`` must not branch on host
values other than the epoch index and must not synchronise (``.item()``) -- the same contract as
CUDA graphs.  A ``train_batch`` that reads ``batch_idx`` at all runs eagerly (checked from its
bytecode by ``reads_argument``, logged once).  Eligibility is checked once: no dynamic loss scaler, every optimizer fused with step-invariant
kernel arguments.  Anything else runs eagerly, logged once.

Data-parallel and aggregation steps are captured too (round 6).  The gradient bucketer's RCCL
collectives (all-reduce, or the fp32_accum all-to-all + det_sum_rows + all-gather on its side
stream) are issued from the capturing stream's backward hooks, so they are recorded into the step's
graph in bucket order and replay overlapped with the backward exactly as they ran eagerly; every
rank replays the same collective sequence whether a given rank replays or runs eagerly (a capture
executes nothing).  With ``aggregation_frequency`` N each position in the window (N - 1 local
backwards, then the communicating one) is its own graph key; a replay runs no Python, so the host
state a step leaves behind -- the GradSink window (fresh / accumulating) and the fused optimizer's
step counters, only for graphs that stepped -- is restored from what the capture recorded, which
lets replayed and eager positions mix inside one window.  The bucket-cap autotuner measures eager
windows: steps stay eager until it has decided.

Multi-batch graphs (``optimizations.hip_graph_batches: K``): even one replay per batch leaves the
CIFAR trial host-bound (data fetch, input copy, replay launch, metric clones: ~0.8 ms/batch against
~0.1 ms of GPU work, ``profiles/r2_asha_baseline_shape_seed1_hipgraph_u8_cl.json``).
``run_chunk`` captures K consecutive ``train_batch`` calls over the K batch views of one
``BatchChunk`` input buffer into ONE graph whose metric outputs are stacked [K] tensors, so the
host cost -- one input copy per leaf, one replay, one clone per metric -- is paid once per K
batches.  Chunks never cross an epoch (the epoch index is part of the key).
"""
import contextlib
import os
import logging
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple

import torch
from torch.utils import _pytree as pytree

WARMUP = 2        # eager batches per key before capturing (lazy init, MIOpen find, allocator)
# "thread_local": other threads may keep calling the HIP API while a step is being captured -- the
# RCCL process group's watchdog thread queries its work events continuously, which "global" mode
# turns into a capture error (hipErrorStreamCaptureUnsupported) and a process abort
CAPTURE_MODE = "thread_local"
MAX_GRAPHS = 2    # live graphs (the epoch's full batch + its tail batch)
THRASH_LIMIT = 8  # captures that replayed fewer than THRASH_MIN times -> graphs off
THRASH_MIN = 4
# Captured steps keep the arena GradSink (ops/arena.py): each window's gradients land in the arena
# through one multi-tensor copy per group instead of one `grad += new` launch per parameter (~180 per
# BERT-base step, 0.9 ms in the r5s20 graph profile).
GRAPH_SINK = os.environ.get("DET_GRAPH_SINK", "1") != "0"
# (debugging) keep the captured hipGraph_t so scripts can list its nodes (scripts/dbg/graph_nodes.py)
KEEP_GRAPH = os.environ.get("DET_GRAPH_KEEP", "0") == "1"
# HIP runtime defect on this stack: a small hipMemsetAsync captured into a graph writes a stale, garbage
# pattern from the graph's second launch on (<= 4 KiB reproduced, 1 MiB fine; scripts/dbg/
# memset_graph_repro.py, profiles/r6_graph_memset_root_cause.txt).  torch's cross-block reductions
# reset their semaphores that way -- e.g. the bias gradient of a bf16 Linear at batch >= 512, which
# froze at its captured value in every later ResNet-50 replay.  Every capture therefore keeps its
# hipGraph_t, has its memset nodes rewritten into fill-kernel nodes (ops/csrc/det_graph.hip), and is
# instantiated after that.  DET_GRAPH_FIX_MEMSETS=0 leaves the graphs as captured.
FIX_MEMSETS = os.environ.get("DET_GRAPH_FIX_MEMSETS", "1") != "0"
MEMSET_FIXES = {"graphs": 0, "memset_nodes": 0}


def new_graph() -> "torch.cuda.CUDAGraph":
    return torch.cuda.CUDAGraph(keep_graph=True) if (KEEP_GRAPH or FIX_MEMSETS) else torch.cuda.CUDAGraph()


def finish_capture(graph: "torch.cuda.CUDAGraph") -> int:
    """After ``torch.cuda.graph(graph)`` exits: rewrite the memset nodes, then instantiate.
    Returns the number of memset nodes rewritten."""
    n = 0
    if FIX_MEMSETS:
        from determined_1_amd.ops import _lib

        n = int(_lib.get_lib().det_graph_fix_memsets(graph.raw_cuda_graph(), 1))
        if n < 0:
            raise RuntimeError(f"hipGraph memset rewrite failed (code {n})")
        MEMSET_FIXES["graphs"] += 1
        MEMSET_FIXES["memset_nodes"] += n
    if FIX_MEMSETS or KEEP_GRAPH:
        graph.instantiate()
    return n


@contextlib.contextmanager
def _native_rng_advance() -> Iterator[None]:
    """Inside a train-step capture: the native dropout kernels (ops/transformer.py) take their
    Philox (seed, offset) as kernel arguments, which a replay repeats; they also add a device offset
    counter, and the captured step starts by bumping it, so every replay draws new masks."""
    from determined_1_amd.ops import transformer as _tf

    c0, existed = _tf.rng_calls(), set(_tf._RNG_BASE)
    _tf.bump_rng_base()
    yield
    if _tf.rng_calls() != c0 and set(_tf._RNG_BASE) != existed:
        # the counter was created inside the capture (its zero-fill would run on every replay): fail
        # this capture; the eager step creates it and the next capture bumps it
        raise RuntimeError("native dropout offset counter created during capture")
CHUNK_WARMUP = 1  # per-batch chunks per multi-batch key before capturing it
CHUNK_MAX_GRAPHS = 8  # full chunks + the partial sizes steps and epochs end on


# Half-precision convolutions on the vendor library (MIOpen) looked replay-unsafe in round 5: a plain
# bf16 torch CNN trained K steps per graph with eager steps in between went NaN on the second replay
# (scripts/dbg/miopen_graph_repro.py --step).  Round 6 pinned the mechanism: MIOpen's weight-gradient
# solvers zero their accumulation buffers with small hipMemsetAsync calls, and a captured small memset
# replays a stale pattern from the graph's second launch on (FIX_MEMSETS above).  With the memset nodes
# rewritten, the same repro replays exactly (profiles/r6_graph_memset_root_cause.txt), so the probe
# below only keeps MIOpen steps eager when the rewrite is turned off (DET_GRAPH_FIX_MEMSETS=0).
# The first warm-up step of EVERY graph key runs under this probe; a hit keeps that key eager (other
# keys still capture).
# DET_GRAPH_LIBRARY_CONVS=1 captures anyway (for the reproduction scripts).
LIBRARY_CONV_OPS = ("aten::convolution", "aten::convolution_backward", "aten::_convolution",
                    "aten::miopen_convolution", "aten::cudnn_convolution")
# torch's dense embedding backward over more than this many indices sorts them and sizes its later
# launches from a segment count read back to the host: a replay keeps the captured batch's sizes and
# a batch with more distinct ids runs out of bounds (the BERT replays faulted in rocprim's
# partition_kernel after ~700 steps, round 5; models/bert.py now uses ops.transformer.bert_embeddings,
# whose backward is shape-sized).  The probe keeps such a train_batch eager.
EMBED_SORT_INDICES = 3072


class _LibraryConvProbe:
    """TorchDispatchMode wrapper that notes the first half-precision convolution a step dispatches to
    the vendor library (torch.backends.cudnn.enabled, a CUDA input in bf16/fp16)."""

    def __init__(self) -> None:
        from torch.utils._python_dispatch import TorchDispatchMode

        probe = self

        class _Mode(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, args=(), kwargs=None):  # noqa: ANN001
                if probe.found is None:
                    name = func.name()
                    if name in LIBRARY_CONV_OPS and torch.backends.cudnn.enabled and not FIX_MEMSETS:
                        x = args[0] if args else None
                        if isinstance(x, torch.Tensor) and x.is_cuda and x.dtype in (torch.bfloat16, torch.float16):
                            probe.found = f"half-precision MIOpen convolution ({name} on {x.dtype})"
                    elif name == "aten::embedding_dense_backward" and len(args) > 1:
                        idx = args[1]
                        if isinstance(idx, torch.Tensor) and idx.is_cuda and idx.numel() > EMBED_SORT_INDICES:
                            probe.found = f"torch embedding backward over {idx.numel()} indices (host-sized sort path)"
                return func(*args, **(kwargs or {}))

        self.found: Optional[str] = None
        self.mode = _Mode()

    def run(self, fn: Callable[[], Any]) -> Any:
        with self.mode:
            return fn()


def library_conv_reason(fn: Callable[[], Any]) -> Tuple[Any, Optional[str]]:
    """Run ``fn`` (one eager step) under the probe: (its result, a reason to stay eager or None)."""
    if os.environ.get("DET_GRAPH_LIBRARY_CONVS", "0") == "1":
        return fn(), None
    probe = _LibraryConvProbe()
    out = probe.run(fn)
    if probe.found is None:
        return out, None
    return out, (f"{probe.found} -- not replay-safe from a captured graph "
                 "(pytorch/_graph.py LIBRARY_CONV_OPS note; DET_GRAPH_LIBRARY_CONVS=1 captures anyway)")


def reads_argument(fn: Callable[..., Any], name: str) -> bool:
    """Whether ``fn``'s body can observe its argument ``name`` (conservatively True when the code is
    not inspectable or it uses locals()/frames).  A ``train_batch`` that never reads ``epoch_idx``
    lets one graph serve every epoch instead of re-capturing at each epoch boundary."""
    import dis
    import inspect

    fn = inspect.unwrap(getattr(fn, "__func__", fn))
    code = getattr(fn, "__code__", None)
    if code is None or name not in code.co_varnames[:code.co_argcount + code.co_kwonlyargcount]:
        return True
    if "locals" in code.co_names or "vars" in code.co_names or "_getframe" in code.co_names:
        return True
    if name in code.co_cellvars:  # captured by a nested function
        return True
    return any(ins.argval == name for ins in dis.get_instructions(code)
               if ins.opname in ("LOAD_FAST", "LOAD_DEREF", "LOAD_CLOSURE", "DELETE_FAST", "STORE_FAST"))


def _leaf_sig(x: Any) -> Any:
    if isinstance(x, torch.Tensor):
        return ("T", tuple(x.shape), x.dtype, x.device.type)
    return ("V", repr(x))


class _Graph:
    def __init__(self, graph: "torch.cuda.CUDAGraph", static_in: List[torch.Tensor], in_spec: Any,
                 out: Any, stepped: Optional[List[int]] = None, sinks_after: Optional[List[bool]] = None) -> None:
        self.graph = graph
        self.static_in = static_in
        self.in_spec = in_spec
        self.out = out
        self.replays = 0
        # per fused optimizer: step() calls the capture recorded (0 for a non-communicating position
        # of an aggregation window), and per GradSink: the window state the captured step left
        self.stepped = stepped
        self.sinks_after = sinks_after


class TrainStepGraph:
    """Per-controller graph cache.  ``run(batch, epoch_idx, batch_idx)`` returns the train_batch
    metrics, eagerly or from a replay."""

    def __init__(self, context: Any, train_batch: Callable[..., Any],
                 epoch_sensitive: Optional[bool] = None) -> None:
        self.context = context
        self.train_batch = train_batch
        # the epoch index is part of the key only when train_batch can read it
        self.epoch_sensitive = reads_argument(train_batch, "epoch_idx") if epoch_sensitive is None \
            else epoch_sensitive
        self.fused = [st.fused for st in context._opt_states if st.fused is not None]
        if not GRAPH_SINK:
            for f in self.fused:  # plain arena accumulation: one `grad += new` launch per parameter
                if f.sink is not None:
                    f.sink.detach()
                    f.sink = None
        self.graphs: Dict[Any, _Graph] = {}
        self.seen: Dict[Any, int] = {}
        self.captures = 0
        self.failed_captures = 0
        self.replays = 0
        self.disabled_reason: Optional[str] = None
        self.pool = None
        self.chunk_graphs: Dict[Any, _Graph] = {}
        self.chunk_disabled: Optional[str] = None
        self.chunk_replays = 0
        self.last_chunk_metrics: Optional[List[Any]] = None
        # graph key -> None (its first warm-up step ran clean under the library-convolution probe) or
        # the reason it stays eager.  Per key, not per controller: another batch shape, an epoch-
        # sensitive key or a new hyper-parameter signature can route to different kernels.
        self.probed: Dict[Any, Optional[str]] = {}

    # ------------------------------------------------------------------------------------------
    @staticmethod
    def ineligible_reason(context: Any) -> Optional[str]:
        if context.device.type != "cuda":
            return "not on a GPU"
        if context._amp is not None and context._amp.scaler is not None:
            return "dynamic loss scaling syncs on overflow"
        if context._timers.enabled:
            return "DET_STEP_TIMERS synchronises the step"
        if not context._opt_states:
            return "no wrapped optimizer"
        for st in context._opt_states:
            if st.fused is None:
                return f"optimizer {type(st.opt).__name__} is not fused"
            if not st.fused.graph_capturable():
                return f"fused {st.fused.kind} changes kernel arguments every step"
        return None

    def _agg(self) -> int:
        return max(1, int(getattr(self.context.dist_config, "aggregation_frequency", 1) or 1))

    def _key(self, leaves: List[Any], epoch_idx: int, batch_idx: int = 0) -> Any:
        # the position in an aggregation window decides which kernels run (local accumulation or
        # the communicating backward + optimizer step): one graph per position
        pos = batch_idx % self._agg() if self._agg() > 1 else None
        return (tuple(_leaf_sig(x) for x in leaves), epoch_idx if self.epoch_sensitive else None,
                tuple(f.graph_signature() for f in self.fused), pos)

    def _max_graphs(self) -> int:
        return MAX_GRAPHS * self._agg()

    def _tuning(self) -> bool:
        """A bucket-cap autotuner still measuring eager windows."""
        for st in getattr(self.context, "_opt_states", []):
            tuner = getattr(getattr(st, "bucketer", None), "_tuner", None)
            if tuner is not None and not tuner.done:
                return True
        return False

    def _sinks(self) -> List[Any]:
        return [f.sink for f in self.fused if f.sink is not None]

    def _eager(self, batch: Any, epoch_idx: int, batch_idx: int) -> Any:
        self.context._current_batch_idx = batch_idx  # chunk batches: the window position of each
        with self.context._autocast():
            return self.train_batch(batch=batch, epoch_idx=epoch_idx, batch_idx=batch_idx)

    def _after_replay(self, g: "_Graph", batches: int = 1) -> None:
        """Host bookkeeping of a replay: optimizer step counters (for the graphs that stepped) and
        the GradSink window state the captured step(s) left."""
        for i, f in enumerate(self.fused):
            for _ in range(g.stepped[i] if g.stepped is not None else batches):
                f.graph_replayed()
        if g.sinks_after is not None:
            for sink, fresh in zip(self._sinks(), g.sinks_after):
                sink.set_host_state(fresh)

    # ------------------------------------------------------------------------------------------
    def run(self, batch: Any, epoch_idx: int, batch_idx: int) -> Any:
        if self.disabled_reason is not None:
            return self._eager(batch, epoch_idx, batch_idx)
        leaves, spec = pytree.tree_flatten(batch)
        if any(isinstance(x, torch.Tensor) and x.device.type != "cuda" for x in leaves):
            self._disable("train batch has host tensors")
            return self._eager(batch, epoch_idx, batch_idx)
        if self._tuning():
            return self._eager(batch, epoch_idx, batch_idx)
        key = self._key(leaves, epoch_idx, batch_idx)
        g = self.graphs.get(key)
        if g is not None:
            return self._replay(g, leaves)
        if self.probed.get(key) is not None:  # this key routes to replay-unsafe kernels: eager
            return self._eager(batch, epoch_idx, batch_idx)
        n = self.seen.get(key, 0) + 1
        self.seen[key] = n
        if key not in self.probed:
            out, reason = library_conv_reason(lambda: self._eager(batch, epoch_idx, batch_idx))
            self.probed[key] = reason
            if reason is not None:
                logging.warning("hip_graph: train_batch runs eagerly for batch signature %s: %s", key[0], reason)
            return out
        if n <= WARMUP:
            return self._eager(batch, epoch_idx, batch_idx)
        g = self._capture(key, leaves, spec, epoch_idx, batch_idx)
        if g is None:
            return self._eager(batch, epoch_idx, batch_idx)
        # the capture recorded but did not execute this batch's work: run it now (host state
        # was advanced during the capture itself)
        for i, f in enumerate(self.fused):
            if g.stepped is None or g.stepped[i]:
                f.graph_prepare(advanced=True)
        g.graph.replay()
        self.replays += 1
        g.replays += 1
        return self._clone_out(g.out)

    def _replay(self, g: _Graph, leaves: List[Any]) -> Any:
        for dst, src in zip(g.static_in, (x for x in leaves if isinstance(x, torch.Tensor))):
            dst.copy_(src, non_blocking=True)
        for i, f in enumerate(self.fused):
            if g.stepped is None or g.stepped[i]:
                f.graph_prepare()
        g.graph.replay()
        self._after_replay(g)
        self.replays += 1
        g.replays += 1
        return self._clone_out(g.out)

    @staticmethod
    def _clone_out(out: Any) -> Any:
        return pytree.tree_map(lambda t: t.detach().clone() if isinstance(t, torch.Tensor) else t, out)

    def _capture(self, key: Any, leaves: List[Any], spec: Any, epoch_idx: int, batch_idx: int) -> Optional[_Graph]:
        stale = [k for k, v in self.graphs.items() if v.replays < THRASH_MIN]
        if self.captures - len(self.graphs) >= THRASH_LIMIT and len(stale) == len(self.graphs):
            self._disable("graph key changes every few batches (per-batch hyper-parameter schedule?)")
            return None
        if len(self.graphs) >= self._max_graphs():
            torch.cuda.synchronize()  # never destroy a graph exec that may still be running
            while len(self.graphs) >= self._max_graphs():
                del self.graphs[next(iter(self.graphs))]
        static_in = [x.detach().clone() for x in leaves if isinstance(x, torch.Tensor)]
        it = iter(static_in)
        static_leaves = [next(it) if isinstance(x, torch.Tensor) else x for x in leaves]
        static_batch = pytree.tree_unflatten(static_leaves, spec)
        host = [f.host_state() for f in self.fused]
        calls0 = [f.steps_called for f in self.fused]
        graph = new_graph()
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        try:
            torch.cuda.synchronize()
            for f in self.fused:
                f.capturing(True)
            try:
                with torch.cuda.graph(graph, pool=self.pool, capture_error_mode=CAPTURE_MODE), _native_rng_advance():
                    out = self._eager(static_batch, epoch_idx, batch_idx)
            finally:
                for f in self.fused:
                    f.capturing(False)
            finish_capture(graph)
        except Exception as e:  # capture-unsafe op in user code or a library: stay eager
            for f, h in zip(self.fused, host):
                f.set_host_state(h)
            self.failed_captures += 1
            self._disable(f"capture failed: {type(e).__name__}: {e}")
            torch.cuda.synchronize()
            return None
        self.captures += 1
        g = _Graph(graph, static_in, spec, out, stepped=[f.steps_called - c for f, c in zip(self.fused, calls0)],
                   sinks_after=[sk.host_state() for sk in self._sinks()])
        self.graphs[key] = g
        return g

    def _disable(self, reason: str) -> None:
        if self.disabled_reason is None:
            logging.warning("hip_graph: running train_batch eagerly: %s", reason)
        self.disabled_reason = reason
        self.graphs.clear()
        self.chunk_graphs.clear()

    # ---- multi-batch graphs ------------------------------------------------------------------
    def run_chunk(self, chunk: Any, epoch_idx: int, batch_idx: int,
                  capture: bool = True) -> Optional[Dict[str, torch.Tensor]]:
        """K train steps over ``chunk`` (a device ``BatchChunk``) as one replay; returns stacked [K]
        metrics, or None when the chunk ran batch by batch (warm-up / ineligible / ``capture``
        False: partial chunks at epoch ends replay per batch rather than growing one multi-batch
        graph per odd size) -- then the per-batch metrics are in ``self.last_chunk_metrics``."""
        self.last_chunk_metrics = None
        if self.chunk_disabled is None and not all(f.chunk_capturable() for f in self.fused):
            self.chunk_disabled = "the optimizer's per-step hyper-parameters hold one step (replaying per batch)"
        if capture and self.disabled_reason is None and self.chunk_disabled is None and not self._tuning():
            leaves, spec = pytree.tree_flatten(chunk.stacked)
            if all(not isinstance(x, torch.Tensor) or x.device.type == "cuda" for x in leaves):
                key = ("chunk", chunk.sizes, self._key(leaves, epoch_idx, batch_idx))
                g = self.chunk_graphs.get(key)
                if g is None and not self._batch_key_clean(chunk, epoch_idx):
                    key = None  # warm up / probe per batch first; a replay-unsafe key stays per batch
                if g is not None:
                    for dst, src in zip(g.static_in, (x for x in leaves if isinstance(x, torch.Tensor))):
                        dst.copy_(src, non_blocking=True)
                    g.graph.replay()
                    self._after_replay(g, len(chunk.sizes))
                    self.replays += 1
                    self.chunk_replays += 1
                    g.replays += 1
                    return self._clone_out(g.out)
                n = self.seen.get(key, 0) + 1 if key is not None else 0
                if key is not None:
                    self.seen[key] = n
                if n > CHUNK_WARMUP:
                    g = self._capture_chunk(key, leaves, spec, chunk.sizes, epoch_idx, batch_idx)
                    if g is not None:
                        g.graph.replay()  # the capture advanced host state but executed nothing
                        self.replays += 1
                        self.chunk_replays += 1
                        g.replays += 1
                        return self._clone_out(g.out)
        outs = []
        for i, b in enumerate(chunk.batches):
            # detached: an eager batch's metrics hold its autograd graph, whose AccumulateGrad nodes
            # (bound to this stream) would break the next capture
            outs.append(pytree.tree_map(lambda t: t.detach() if isinstance(t, torch.Tensor) else t,
                                        self.run(b, epoch_idx, batch_idx + i)))
        self.last_chunk_metrics = outs
        return None

    def _batch_key_clean(self, chunk: Any, epoch_idx: int) -> bool:
        """Whether the per-batch graph key of the chunk's first batch probed clean."""
        bl, _ = pytree.tree_flatten(chunk.batches[0])
        k = self._key(bl, epoch_idx, self.context._current_batch_idx or 0)
        return k in self.probed and self.probed[k] is None

    def _capture_chunk(self, key: Any, leaves: List[Any], spec: Any, sizes: Tuple[int, ...], epoch_idx: int,
                       batch_idx: int) -> Optional[_Graph]:
        from determined_1_amd.pytorch._data import BatchChunk

        if len(self.chunk_graphs) >= CHUNK_MAX_GRAPHS:
            torch.cuda.synchronize()  # never destroy a graph exec that may still be running
            while len(self.chunk_graphs) >= CHUNK_MAX_GRAPHS:
                del self.chunk_graphs[next(iter(self.chunk_graphs))]
        static_in = [x.detach().clone() for x in leaves if isinstance(x, torch.Tensor)]
        it = iter(static_in)
        views = BatchChunk(pytree.tree_unflatten([next(it) if isinstance(x, torch.Tensor) else x for x in leaves],
                                                 spec), sizes).batches
        host = [f.host_state() for f in self.fused]
        calls0 = [f.steps_called for f in self.fused]
        graph = new_graph()
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        try:
            torch.cuda.synchronize()
            with torch.cuda.graph(graph, pool=self.pool, capture_error_mode=CAPTURE_MODE), _native_rng_advance():
                outs = []
                for i, b in enumerate(views):
                    o = self._eager(b, epoch_idx, batch_idx + i)
                    o = {"loss": o} if isinstance(o, torch.Tensor) else o
                    if not isinstance(o, dict) or not all(isinstance(v, torch.Tensor) and v.dim() == 0
                                                          for v in o.values()):
                        raise TypeError("train_batch metrics are not all scalar tensors")
                    outs.append(o)
                names = list(outs[0].keys())
                if any(list(o.keys()) != names for o in outs):
                    raise TypeError("train_batch metric names differ between batches")
                out = {k: torch.stack([o[k].detach().float() for o in outs]) for k in names}
            finish_capture(graph)
        except Exception as e:  # noqa: BLE001 - stay on per-batch replays
            for f, h in zip(self.fused, host):
                f.set_host_state(h)
            self.chunk_disabled = f"{type(e).__name__}: {e}"
            logging.warning("hip_graph: multi-batch capture failed, replaying per batch: %s", self.chunk_disabled)
            torch.cuda.synchronize()
            return None
        self.captures += 1
        g = _Graph(graph, static_in, spec, out, stepped=[f.steps_called - c for f, c in zip(self.fused, calls0)],
                   sinks_after=[sk.host_state() for sk in self._sinks()])
        self.chunk_graphs[key] = g
        return g

    def stats(self) -> Dict[str, Any]:
        return {"captures": self.captures, "replays": self.replays, "failed_captures": self.failed_captures,
                "disabled": self.disabled_reason, "chunk_replays": self.chunk_replays,
                "chunk_disabled": self.chunk_disabled, "memset_nodes_rewritten": MEMSET_FIXES["memset_nodes"]}


class EvalStepGraph:
    """``evaluate_batch`` replayed as a hipGraph: no optimizer state, so the key is just the input
    leaves; one eager batch per key (lazy init), then capture.  The validation pass of the ASHA
    benchmark's CIFAR trial runs once per epoch over 10k records."""

    WARMUP = 1

    def __init__(self, context: Any, evaluate_batch: Callable[..., Any]) -> None:
        self.context = context
        self.evaluate_batch = evaluate_batch
        self.graphs: Dict[Any, _Graph] = {}
        self.seen: Dict[Any, int] = {}
        self.pool = None
        self.disabled_reason: Optional[str] = None
        self.captures = 0
        self.replays = 0
        self.probed: Dict[Any, Optional[str]] = {}

    def _eager(self, batch: Any) -> Any:
        with self.context._autocast():
            return self.evaluate_batch(batch=batch)

    def run(self, batch: Any) -> Any:
        if self.disabled_reason is not None:
            return self._eager(batch)
        leaves, spec = pytree.tree_flatten(batch)
        if any(isinstance(x, torch.Tensor) and x.device.type != "cuda" for x in leaves):
            self.disabled_reason = "evaluation batch has host tensors"
            return self._eager(batch)
        key = tuple(_leaf_sig(x) for x in leaves)
        g = self.graphs.get(key)
        if g is None:
            n = self.seen.get(key, 0) + 1
            self.seen[key] = n
            if self.probed.get(key) is not None:
                return self._eager(batch)
            if key not in self.probed:  # every key's first batch under the probe (as TrainStepGraph)
                out, reason = library_conv_reason(lambda: self._eager(batch))
                self.probed[key] = reason
                if reason is not None:
                    logging.warning("hip_graph: evaluate_batch runs eagerly for batch signature %s: %s", key, reason)
                return out
            if n <= self.WARMUP:
                return self._eager(batch)
            if len(self.graphs) >= MAX_GRAPHS:
                torch.cuda.synchronize()
                while len(self.graphs) >= MAX_GRAPHS:
                    del self.graphs[next(iter(self.graphs))]
            static_in = [x.detach().clone() for x in leaves if isinstance(x, torch.Tensor)]
            it = iter(static_in)
            static_batch = pytree.tree_unflatten([next(it) if isinstance(x, torch.Tensor) else x for x in leaves], spec)
            graph = new_graph()
            if self.pool is None:
                self.pool = torch.cuda.graph_pool_handle()
            try:
                torch.cuda.synchronize()
                with torch.cuda.graph(graph, pool=self.pool, capture_error_mode=CAPTURE_MODE):
                    out = self._eager(static_batch)
                finish_capture(graph)
            except Exception as e:
                logging.warning("hip_graph: evaluate_batch runs eagerly: capture failed: %s: %s", type(e).__name__, e)
                self.disabled_reason = f"capture failed: {e}"
                torch.cuda.synchronize()
                return self._eager(batch)
            self.captures += 1
            g = self.graphs[key] = _Graph(graph, static_in, spec, out)
        else:
            for dst, src in zip(g.static_in, (x for x in leaves if isinstance(x, torch.Tensor))):
                dst.copy_(src, non_blocking=True)
        g.graph.replay()
        self.replays += 1
        return TrainStepGraph._clone_out(g.out)

    def run_chunk(self, chunk: Any) -> Optional[Dict[str, torch.Tensor]]:
        """``evaluate_batch`` over the K batches of a device ``BatchChunk`` as one replay -> stacked
        [K] metrics; None when it ran per batch (metrics in ``last_chunk_metrics``)."""
        from determined_1_amd.pytorch._data import BatchChunk

        self.last_chunk_metrics = None
        leaves, spec = pytree.tree_flatten(chunk.stacked)
        if self.disabled_reason is None and getattr(self, "chunk_disabled", None) is None and \
                all(not isinstance(x, torch.Tensor) or x.device.type == "cuda" for x in leaves):
            key = ("chunk", chunk.sizes, tuple(_leaf_sig(x) for x in leaves))
            g = self.graphs.get(key)
            bkey = tuple(_leaf_sig(x) for x in pytree.tree_flatten(chunk.batches[0])[0])
            clean = bkey in self.probed and self.probed[bkey] is None  # per-batch key probed clean
            if g is None and self.seen.get(key, 0) >= self.WARMUP and clean:
                if len(self.graphs) >= CHUNK_MAX_GRAPHS:
                    torch.cuda.synchronize()
                    while len(self.graphs) >= CHUNK_MAX_GRAPHS:
                        del self.graphs[next(iter(self.graphs))]
                static_in = [x.detach().clone() for x in leaves if isinstance(x, torch.Tensor)]
                it = iter(static_in)
                views = BatchChunk(pytree.tree_unflatten([next(it) if isinstance(x, torch.Tensor) else x
                                                          for x in leaves], spec), chunk.sizes).batches
                graph = new_graph()
                if self.pool is None:
                    self.pool = torch.cuda.graph_pool_handle()
                try:
                    torch.cuda.synchronize()
                    with torch.cuda.graph(graph, pool=self.pool, capture_error_mode=CAPTURE_MODE):
                        outs = [self._eager(b) for b in views]
                        if not all(isinstance(o, dict) and all(isinstance(v, torch.Tensor) and v.dim() == 0
                                                               for v in o.values()) for o in outs):
                            raise TypeError("evaluate_batch metrics are not all scalar tensors")
                        out = {k: torch.stack([o[k].detach().float() for o in outs]) for k in outs[0]}
                    finish_capture(graph)
                except Exception as e:  # noqa: BLE001
                    self.chunk_disabled = f"{type(e).__name__}: {e}"
                    logging.warning("hip_graph: multi-batch evaluate capture failed: %s", self.chunk_disabled)
                    torch.cuda.synchronize()
                    g = None
                else:
                    self.captures += 1
                    g = self.graphs[key] = _Graph(graph, static_in, spec, out)
            else:
                self.seen[key] = self.seen.get(key, 0) + 1
                if g is not None:
                    for dst, src in zip(g.static_in, (x for x in leaves if isinstance(x, torch.Tensor))):
                        dst.copy_(src, non_blocking=True)
            if g is not None:
                g.graph.replay()
                self.replays += 1
                return TrainStepGraph._clone_out(g.out)
        self.last_chunk_metrics = [self.run(b) for b in chunk.batches]
        return None


def build(context: Any, train_batch: Callable[..., Any], enabled: bool,
          epoch_sensitive: Optional[bool] = None) -> Tuple[Optional[TrainStepGraph], Optional[str]]:
    if not enabled:
        return None, None
    reason = TrainStepGraph.ineligible_reason(context)
    if reason is None and reads_argument(train_batch, "batch_idx"):
        # a replay re-runs the captured kernels with the batch_idx of the capture: a train_batch
        # that branches on it (or feeds it to a kernel) would train silently wrong
        reason = "train_batch reads batch_idx (a graph replay would reuse the captured value)"
    if reason is not None:
        logging.warning("optimizations.hip_graph is set but train_batch will run eagerly: %s", reason)
        return None, reason
    return TrainStepGraph(context, train_batch, epoch_sensitive), None
