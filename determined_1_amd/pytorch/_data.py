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
"""
import logging
from typing import Any, Callable, Dict, Iterator, List, Optional, Sequence, Set, Type, Union

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
