"""Data loading for PyTorchTrial (reference ``harness/determined/pytorch/_data.py``).

``DataLoader`` is a *lazy spec* with torch's DataLoader constructor signature: the controller
calls ``get_data_loader(repeat, skip, num_replicas, rank)`` to build the real loader with the
sampler stack of SURVEY C-data:

    BatchSampler -> Repeat (training) -> DistributedBatchSampler (every num_replicas-th batch
    starting at rank) -> SkipBatchSampler (skip already-trained batches after a restore)

The skip is counted in *sharded* batches, applied after sharding (reference ``_data.py:221-246``).

MI355X addition: ``DevicePrefetcher`` moves the next batches host->device on a side HIP stream
(pinned memory, non_blocking copies) so the H2D transfer of batch k+1 overlaps compute of batch
k instead of stalling the training stream (the reference copies synchronously in the loop).

Batch chunks (``optimizations.hip_graph_batches``): for datasets whose ``__getitems__`` returns
stacked rows (``collate_fn=passthrough_collate``), ``ChunkedBatches`` fetches K consecutive
batches with ONE dataset call and ``ChunkPrefetcher`` moves them with one pinned H2D copy per
leaf, so a small model's per-batch host cost (sampler, dataset call, pinning, copy, event) is paid
once per K batches; the trial controller then replays K train steps as one hipGraph.
"""
import logging
from typing import Any, Callable, Dict, Iterator, List, Optional, Sequence, Set, Tuple, Type, Union

import numpy as np
import torch
import torch.utils.data as tud

_Array = Union[np.ndarray, torch.Tensor]
_Data = Union[Dict[str, _Array], Sequence[_Array], _Array]
TorchData = Union[Dict[str, torch.Tensor], Sequence[torch.Tensor], torch.Tensor]


class DataLoader:
    """Lazy DataLoader specification (same constructor as ``torch.utils.data.DataLoader``)."""

    def __init__(
        self,
        dataset: tud.Dataset,
        batch_size: Optional[int] = 1,
        shuffle: bool = False,
        sampler: Optional[tud.Sampler] = None,
        batch_sampler: Optional[tud.BatchSampler] = None,
        num_workers: int = 0,
        collate_fn: Optional[Callable] = None,
        pin_memory: bool = False,
        drop_last: bool = False,
        timeout: float = 0,
        worker_init_fn: Optional[Callable] = None,
        multiprocessing_context: Any = None,
        generator: Any = None,
        prefetch_factor: Optional[int] = None,
        persistent_workers: bool = False,
    ) -> None:
        if isinstance(dataset, tud.IterableDataset):
            raise ValueError("determined DataLoader does not support IterableDataset (it must be indexable)")
        if timeout < 0:
            raise ValueError("timeout option should be non-negative")
        if batch_sampler is not None:
            if batch_size != 1 or shuffle or sampler is not None or drop_last:
                raise ValueError("batch_sampler option is mutually exclusive with batch_size, shuffle, sampler, "
                                 "and drop_last")
            batch_size = None
            drop_last = False
        elif batch_size is None:
            raise ValueError("batch_size=None (auto-collation off) is not supported")
        if sampler is not None and shuffle:
            raise ValueError("sampler option is mutually exclusive with shuffle")
        if sampler is None:
            sampler = tud.RandomSampler(dataset, generator=generator) if shuffle else tud.SequentialSampler(dataset)
        if batch_sampler is None:
            batch_sampler = tud.BatchSampler(sampler, batch_size, drop_last)
        self.dataset = dataset
        self.batch_size = batch_size
        self.sampler = sampler
        self.batch_sampler = batch_sampler
        self.num_workers = num_workers
        self.collate_fn = collate_fn if collate_fn is not None else tud.default_collate
        self.pin_memory = pin_memory
        self.drop_last = drop_last
        self.timeout = timeout
        self.worker_init_fn = worker_init_fn
        self.multiprocessing_context = multiprocessing_context
        self.prefetch_factor = prefetch_factor
        self.persistent_workers = persistent_workers

    def get_data_loader(self, repeat: bool = False, skip: int = 0, num_replicas: int = 1,
                        rank: int = 0) -> tud.DataLoader:
        bs = adapt_batch_sampler(self.batch_sampler, repeat=repeat, skip=skip, num_replicas=num_replicas, rank=rank)
        kwargs = {}  # type: Dict[str, Any]
        if self.num_workers > 0:
            if self.prefetch_factor is not None:
                kwargs["prefetch_factor"] = self.prefetch_factor
            kwargs["persistent_workers"] = self.persistent_workers
            kwargs["multiprocessing_context"] = self.multiprocessing_context
        return tud.DataLoader(
            self.dataset,
            batch_sampler=bs,
            num_workers=self.num_workers,
            collate_fn=self.collate_fn,
            pin_memory=self.pin_memory,
            timeout=self.timeout,
            worker_init_fn=self.worker_init_fn,
            **kwargs,
        )

    def __iter__(self) -> Iterator:
        return iter(self.get_data_loader())

    def __len__(self) -> int:
        return len(self.batch_sampler)


def adapt_batch_sampler(batch_sampler: Any, repeat: bool = False, skip: int = 0, num_replicas: int = 1,
                        rank: int = 0) -> Any:
    if repeat:
        batch_sampler = RepeatBatchSampler(batch_sampler)
    if num_replicas > 1:
        batch_sampler = DistributedBatchSampler(batch_sampler, num_replicas, rank)
    if skip > 0:
        batch_sampler = SkipBatchSampler(batch_sampler, skip, same_length=repeat)
    return batch_sampler


class RepeatBatchSampler(tud.Sampler):
    """Yield the wrapped sampler's batches forever; ``len`` is one pass."""

    def __init__(self, batch_sampler: Any) -> None:
        self.batch_sampler = batch_sampler

    def __len__(self) -> int:
        return len(self.batch_sampler)

    def __iter__(self) -> Iterator:
        while True:
            yield from self.batch_sampler


class DistributedBatchSampler(tud.Sampler):
    """Pass every ``num_replicas``-th batch to this worker, starting at ``rank``."""

    def __init__(self, batch_sampler: Any, num_replicas: int, rank: int) -> None:
        if rank < 0:
            raise ValueError("rank must be non-negative")
        if num_replicas <= 0:
            raise ValueError("num_replicas must be positive")
        if rank >= num_replicas:
            raise ValueError("rank must be less than num_replicas")
        self.batch_sampler = batch_sampler
        self.num_replicas = num_replicas
        self.rank = rank

    def __len__(self) -> int:
        n = len(self.batch_sampler)
        return n // self.num_replicas + int(n % self.num_replicas > self.rank)

    def __iter__(self) -> Iterator:
        if self.num_replicas == 1:
            yield from self.batch_sampler
            return
        for i, b in enumerate(self.batch_sampler):
            if i % self.num_replicas == self.rank:
                yield b


class SkipBatchSampler(tud.Sampler):
    """Skip the first ``skip`` batches; ``len`` excludes them unless ``same_length``."""

    def __init__(self, batch_sampler: Any, skip: int, same_length: bool = False) -> None:
        self.batch_sampler = batch_sampler
        self.skip = skip
        self.length = len(batch_sampler) - (0 if same_length else skip)

    def __len__(self) -> int:
        return self.length

    def __iter__(self) -> Iterator:
        it = iter(self.batch_sampler)
        for _ in range(self.skip):
            try:
                next(it)
            except StopIteration:
                return
        yield from it


def passthrough_collate(batch: Any) -> Any:
    """Collate for datasets whose ``__getitems__`` already returns a stacked batch.  Contract (what
    makes batch chunking valid): ``__getitems__(idx)`` returns rows that depend only on their own
    index, stacked along dim 0 of every leaf."""
    return batch


def stacked_rows_loader(loader: Any) -> bool:
    """Whether a built torch DataLoader can be fetched K batches per dataset call."""
    return (getattr(loader, "num_workers", 1) == 0 and getattr(loader, "collate_fn", None) is passthrough_collate
            and hasattr(loader.dataset, "__getitems__") and getattr(loader, "batch_sampler", None) is not None)


def _split_rows(data: Any, sizes: Sequence[int]) -> List[Any]:
    """Per-batch dim-0 views of a stacked batch."""
    if isinstance(data, np.ndarray):
        data = torch.from_numpy(data)
    if isinstance(data, torch.Tensor):
        return list(torch.split(data, list(sizes)))
    if isinstance(data, dict):
        parts = {k: _split_rows(v, sizes) for k, v in data.items()}
        return [{k: parts[k][i] for k in data} for i in range(len(sizes))]
    if isinstance(data, (list, tuple)):
        parts = [_split_rows(v, sizes) for v in data]
        return [type(data)(p[i] for p in parts) for i in range(len(sizes))]
    return [data] * len(sizes)


class BatchChunk:
    """K consecutive batches: ``stacked`` (every leaf holds the K batches' rows back to back),
    ``sizes`` (rows per batch) and ``batches`` (per-batch views, built on first use)."""

    def __init__(self, stacked: Any, sizes: Sequence[int]) -> None:
        self.stacked = stacked
        self.sizes = tuple(sizes)
        self._batches = None  # type: Optional[List[Any]]

    def __len__(self) -> int:
        return len(self.sizes)

    @property
    def batches(self) -> List[Any]:
        if self._batches is None:
            self._batches = _split_rows(self.stacked, self.sizes)
        return self._batches

    def split(self, r: int) -> Tuple["BatchChunk", "BatchChunk"]:
        """(first r batches, the rest) as chunks over row views of the same storage."""
        rows = sum(self.sizes[:r])
        total = sum(self.sizes)
        head, tail = _split_rows(self.stacked, [rows, total - rows])
        return BatchChunk(head, self.sizes[:r]), BatchChunk(tail, self.sizes[r:])


class ChunkedBatches:
    """Iterator of ``BatchChunk``: up to ``k`` batches of ``loader.batch_sampler`` per ONE
    ``dataset.__getitems__`` call.  Chunks never cross an epoch boundary (``epoch_len`` batches
    from batch index 0; the iterator starts at batch ``start``), so every batch of a chunk shares
    its epoch index, nor a multiple of ``unit`` batches after ``start`` (the scheduling unit: the
    training steps a container runs), so a step ends on a chunk boundary."""

    def __init__(self, loader: Any, k: int, epoch_len: Optional[int] = None, start: int = 0,
                 unit: Optional[int] = None) -> None:
        self.dataset = loader.dataset
        self._it = iter(loader.batch_sampler)
        self.k = max(1, int(k))
        self.epoch_len = epoch_len
        self.unit = unit
        self.start = start
        self.next_idx = start

    def __iter__(self) -> "ChunkedBatches":
        return self

    def __next__(self) -> BatchChunk:
        n = self.k
        if self.epoch_len:
            n = min(n, self.epoch_len - self.next_idx % self.epoch_len)
        if self.unit:
            n = min(n, self.unit - (self.next_idx - self.start) % self.unit)
        idx = []  # type: List[int]
        sizes = []  # type: List[int]
        for _ in range(n):
            try:
                b = next(self._it)
            except StopIteration:
                break
            b = list(b)
            idx.extend(b)
            sizes.append(len(b))
        if not sizes:
            raise StopIteration
        self.next_idx += len(sizes)
        return BatchChunk(self.dataset.__getitems__(idx), sizes)


def data_length(data: _Data) -> int:
    """Batch size of a (possibly nested) batch: length of the first array/tensor leaf."""
    if isinstance(data, (np.ndarray, torch.Tensor)):
        return len(data)
    if isinstance(data, dict):
        if not data:
            raise ValueError("`PyTorchTrial` must have at least one `np.ndarray` or `torch.Tensor` in its dict of inputs.")
        return data_length(next(iter(data.values())))
    if isinstance(data, (list, tuple)):
        if not data:
            raise ValueError("`PyTorchTrial` must have at least one `np.ndarray` or `torch.Tensor` in its inputs.")
        return data_length(data[0])
    raise TypeError(f"Data of incorrect type: {type(data)}")


def to_device(data: _Data, device: torch.device, warned_types: Optional[Set[Type]] = None,
              non_blocking: bool = False) -> TorchData:
    """Recursively move arrays/tensors (and objects with ``.to``) to ``device``."""
    if warned_types is None:
        warned_types = set()
    if isinstance(data, dict):
        return {k: to_device(v, device, warned_types, non_blocking) for k, v in data.items()}  # type: ignore
    if isinstance(data, list):
        return [to_device(d, device, warned_types, non_blocking) for d in data]  # type: ignore
    if isinstance(data, tuple):
        return tuple(to_device(d, device, warned_types, non_blocking) for d in data)  # type: ignore
    if isinstance(data, np.ndarray):
        return torch.from_numpy(data).to(device, non_blocking=non_blocking)
    if isinstance(data, torch.Tensor):
        return data.to(device, non_blocking=non_blocking)
    if hasattr(data, "to") and callable(data.to):
        return data.to(device)  # type: ignore
    if type(data) not in warned_types:
        warned_types.add(type(data))
        logging.warning(f"Was not able to move data item of type '{type(data).__name__}' to device.")
    return data  # type: ignore


def _pin(data: Any) -> Any:
    if isinstance(data, torch.Tensor):
        return data if data.is_pinned() else data.pin_memory()
    if isinstance(data, np.ndarray):
        return torch.from_numpy(data).pin_memory()
    if isinstance(data, dict):
        return {k: _pin(v) for k, v in data.items()}
    if isinstance(data, (list, tuple)):
        return type(data)(_pin(v) for v in data)
    return data


def _record_stream(data: Any, stream: Any) -> None:
    if isinstance(data, torch.Tensor):
        data.record_stream(stream)
    elif isinstance(data, dict):
        for v in data.values():
            _record_stream(v, stream)
    elif isinstance(data, (list, tuple)):
        for v in data:
            _record_stream(v, stream)


def shutdown_iterator(it: Any) -> None:
    """Stop the worker processes behind a (wrapped) torch DataLoader iterator.  A trial's training
    iterator repeats forever, so torch never reaches the end that shuts its workers down; left to
    the garbage collector, the shutdown (a join per worker) lands inside whatever runs next."""
    for _ in range(4):
        if it is None:
            return
        stop = getattr(it, "_shutdown_workers", None)
        if callable(stop):
            stop()
            return
        it = getattr(it, "_it", None)


class DevicePrefetcher:
    """Iterator adaptor: pulls host batches (collation happens in DataLoader workers when
    ``num_workers > 0``) and issues their pinned H2D copies on a dedicated HIP stream ``depth``
    batches ahead.  Each yielded batch is already on
    ``device`` and ordered before use on the consumer's current stream (event wait, no host
    sync).  Yields ``(host_batch_len, device_batch)``.
    """

    def __init__(self, iterator: Iterator, device: torch.device, depth: int = 2) -> None:
        self._it = iterator
        self._device = device
        self._depth = max(1, depth)
        self._stream = torch.cuda.Stream(device=device) if device.type == "cuda" else None
        self._queue = []  # type: List[Any]
        self._warned = set()  # type: Set[Type]

    def _fetch_one(self) -> None:
        host = next(self._it)
        n = data_length(host)
        if self._stream is None:
            self._queue.append((n, to_device(host, self._device, self._warned), None))
            return
        host = _pin(host)
        with torch.cuda.stream(self._stream):
            dev = to_device(host, self._device, self._warned, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        self._queue.append((n, dev, ev))

    def __iter__(self) -> "DevicePrefetcher":
        return self

    def __next__(self) -> Any:
        while len(self._queue) < self._depth:
            try:
                self._fetch_one()
            except StopIteration:
                break
        if not self._queue:
            raise StopIteration
        n, dev, ev = self._queue.pop(0)
        if ev is not None:
            cur = torch.cuda.current_stream(self._device)
            cur.wait_event(ev)
            _record_stream(dev, cur)
        return n, dev


class ChunkPrefetcher:
    """``DevicePrefetcher`` for ``BatchChunk`` streams: one pinned H2D copy per leaf per chunk on a
    side stream, ``depth`` chunks ahead, from a reused ring of pinned staging buffers (no
    per-batch ``pin_memory`` allocation).  Yields device ``BatchChunk``s ordered on the consumer's
    current stream.  On the CPU it yields the host chunks unchanged."""

    def __init__(self, chunks: Iterator[BatchChunk], device: torch.device, depth: int = 2) -> None:
        self._it = chunks
        self._device = device
        self._depth = max(1, depth)
        self._cuda = device.type == "cuda"
        self._stream = torch.cuda.Stream(device=device) if self._cuda else None
        self._queue = []  # type: List[Any]
        self._ring = []  # type: List[Any]  # (leaf signature, pinned leaves, event) per slot
        self._slot = 0

    def _stage(self, leaves: List[torch.Tensor]) -> List[torch.Tensor]:
        sig = [(tuple(t.shape), t.dtype) for t in leaves]
        if len(self._ring) < self._depth + 1:
            self._ring.append(None)
        slot = self._slot
        self._slot = (self._slot + 1) % (self._depth + 1)
        ent = self._ring[slot]
        if ent is not None:
            ent[2].synchronize()  # the copy that last read this slot (normally long done)
        if ent is None or ent[0] != sig:
            ent = [sig, [torch.empty(t.shape, dtype=t.dtype).pin_memory() for t in leaves], None]
            self._ring[slot] = ent
        for dst, src in zip(ent[1], leaves):
            dst.copy_(src)
        return ent

    def _fetch_one(self) -> None:
        from torch.utils import _pytree as pytree

        c = next(self._it)
        if not self._cuda:
            self._queue.append((c, None))
            return
        leaves, spec = pytree.tree_flatten(c.stacked)
        tensors = [torch.from_numpy(x) if isinstance(x, np.ndarray) else x for x in leaves]
        is_t = [isinstance(x, torch.Tensor) for x in tensors]
        ent = self._stage([x for x, t in zip(tensors, is_t) if t])
        with torch.cuda.stream(self._stream):
            it = iter(ent[1])
            dev = [next(it).to(self._device, non_blocking=True) if t else x for x, t in zip(tensors, is_t)]
            ev = torch.cuda.Event()
            ev.record(self._stream)
        ent[2] = ev
        self._queue.append((BatchChunk(pytree.tree_unflatten(dev, spec), c.sizes), ev))

    def __iter__(self) -> "ChunkPrefetcher":
        return self

    def __next__(self) -> BatchChunk:
        while len(self._queue) < self._depth:
            try:
                self._fetch_one()
            except StopIteration:
                break
        if not self._queue:
            raise StopIteration
        c, ev = self._queue.pop(0)
        if ev is not None:
            cur = torch.cuda.current_stream(self._device)
            cur.wait_event(ev)
            _record_stream(c.stacked, cur)
        return c
