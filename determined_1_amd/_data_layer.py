"""Dataset cache for PyTorch trials (reference ``harness/determined/_data_layer/_data_layer.py:33-217``
and ``_context.py``; the reference is tf.data + yogadl, this one is map-style PyTorch datasets).

``context.experimental.cache_train_dataset(id, version, shuffle=...)`` decorates a function that
builds a map-style dataset (``__len__`` + ``__getitem__`` returning a tensor/ndarray, a tuple of
them, or a dict of them).  The first caller materialises every sample once into a column store::

    <storage>/<dataset_id>/<dataset_version>_{train,val}/meta.json + col_<k>.npy

(one contiguous ``.npy`` per field, written to a temp dir and renamed in, so readers never see a
partial cache).  Later calls -- other ranks, restarts, other trials of the experiment -- memory-map
the columns instead of re-running the (usually expensive) decode/pre-processing.

Storage types (reference ``data_layer`` config): ``shared_fs`` (the cache lives under
``container_storage_path``), and ``s3`` / ``gcs`` (reference yogadl's S3/GCS storage): the cache is
written locally, uploaded under ``<bucket>/<bucket_directory_path>/<id>/<version>/`` with
``meta.json`` last, and other nodes download it into ``local_cache_path`` instead of rebuilding it
(object-store REST clients of ``storage/rest_clients.py``; no SDKs).

The writer holds an exclusive lock and readers a shared one: through the master's RW coordinator
(WS ``/ws/data-layer/*``, ``native/src/rw_coordinator.cc``) when the trial runs under a master, and
an ``fcntl`` file lock in local mode.

Exactly ONE layer owns sharding, shuffling and resume, depending on who consumes the data:
  * PyTorchTrial (``map_style=True``, what ``PyTorchTrialContext.experimental`` uses): the decorated
    function returns the map-style :class:`CachedDataset`.  The user wraps it in
    ``det.pytorch.DataLoader`` as with any dataset, and the controller's sampler stack
    (Repeat -> DistributedBatchSampler -> SkipBatchSampler, ``pytorch/_data.py``) shards it and
    skips the batches a restored trial already trained on.  ``shuffle=True`` applies one fixed
    permutation seeded by the trial seed (``skip_shuffle_at_epoch_end`` semantics); per-epoch
    reshuffling is ``DataLoader(shuffle=True)``'s job, as for any map-style dataset.
  * other consumers (native loops, ``map_style=False``): a :class:`CachedStream`, an
    ``IterableDataset`` that shards (``rank::size``), shuffles with the trial seed (reshuffled per
    epoch unless ``skip_shuffle_at_epoch_end``) and starts ``total_batches_processed * per_slot``
    samples in, so a resumed trial continues where its checkpoint left off.  Training streams repeat
    forever; validation streams are one pass without dropping the shard remainder.
"""
import contextlib
import fcntl
import functools
import json
import logging
import os
import pathlib
import shutil
import tempfile
from typing import Any, Callable, Dict, Iterator, List, Optional

import numpy as np
import torch

SUPPORTED_TYPES = ("shared_fs", "s3", "gcs")


def init_container_storage_path(configured: Optional[str]) -> pathlib.Path:
    """Reference ``_data_layer.py:17-24``: the configured path, default ``~/data/determined``; falls
    back to a per-user temp dir where that is not writable."""
    path = pathlib.Path(configured) if configured else pathlib.Path.home().joinpath("data/determined")
    try:
        path.mkdir(parents=True, exist_ok=True)
        if not os.access(path, os.W_OK):
            raise PermissionError(str(path))
    except OSError:
        path = pathlib.Path(tempfile.gettempdir()) / f"det_data_layer_{os.getuid()}"
        path.mkdir(parents=True, exist_ok=True)
    return path


def _to_numpy(x: Any) -> np.ndarray:
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def _flatten(sample: Any):
    if isinstance(sample, dict):
        keys = sorted(sample)
        return "dict", keys, [_to_numpy(sample[k]) for k in keys]
    if isinstance(sample, (tuple, list)):
        return "tuple", None, [_to_numpy(v) for v in sample]
    return "single", None, [_to_numpy(sample)]


def remove_stale_temp_dirs(path: pathlib.Path) -> int:
    """Delete ``.tmp_*`` siblings a killed writer left next to ``path`` (call under the write lock)."""
    n = 0
    parent = path.parent
    if not parent.is_dir():
        return 0
    for p in parent.iterdir():
        if p.name.startswith(".tmp_") and p.is_dir():
            shutil.rmtree(str(p), ignore_errors=True)
            n += 1
    return n


def write_cache(dataset: Any, path: pathlib.Path) -> None:
    n = len(dataset)
    if n == 0:
        raise ValueError("cannot cache an empty dataset")
    kind, keys, first = _flatten(dataset[0])
    tmp = pathlib.Path(tempfile.mkdtemp(prefix=".tmp_", dir=str(path.parent)))
    try:
        cols = [np.lib.format.open_memmap(str(tmp / f"col_{k}.npy"), mode="w+", dtype=a.dtype, shape=(n,) + a.shape)
                for k, a in enumerate(first)]
        for i in range(n):
            _, _, arrays = _flatten(dataset[i]) if i else (kind, keys, first)
            if len(arrays) != len(cols):
                raise ValueError(f"sample {i} has {len(arrays)} fields, sample 0 has {len(cols)}")
            for c, a in zip(cols, arrays):
                c[i] = a
        for c in cols:
            c.flush()
        del cols
        meta = {"length": n, "kind": kind, "keys": keys, "num_fields": len(first)}
        (tmp / "meta.json").write_text(json.dumps(meta))
        os.replace(tmp, path)
    finally:
        if tmp.exists():
            shutil.rmtree(tmp, ignore_errors=True)


class CachedDataset(torch.utils.data.Dataset):
    """Random access over a written cache (memory-mapped columns).  ``order`` (optional) is a fixed
    index permutation applied to ``__getitem__`` (the decorator's ``shuffle=True`` in map style)."""

    def __init__(self, path: pathlib.Path, order: Optional[np.ndarray] = None) -> None:
        self.path = path
        self.meta = json.loads((path / "meta.json").read_text())
        self._cols: Optional[List[np.ndarray]] = None
        self.order = order

    def _columns(self) -> List[np.ndarray]:
        if self._cols is None:  # opened lazily so DataLoader workers map the file themselves
            self._cols = [np.load(str(self.path / f"col_{k}.npy"), mmap_mode="r")
                          for k in range(self.meta["num_fields"])]
        return self._cols

    def __getstate__(self) -> Dict[str, Any]:
        return {"path": self.path, "meta": self.meta, "_cols": None, "order": self.order}

    def __len__(self) -> int:
        return int(self.meta["length"])

    def __getitem__(self, i: int) -> Any:
        if self.order is not None:
            i = int(self.order[i])
        vals = [torch.from_numpy(np.array(c[i])) for c in self._columns()]
        if self.meta["kind"] == "dict":
            return dict(zip(self.meta["keys"], vals))
        if self.meta["kind"] == "tuple":
            return tuple(vals)
        return vals[0]


class CachedStream(torch.utils.data.IterableDataset):
    """Sharded, shuffled, offset stream over a :class:`CachedDataset` (yogadl ``Stream`` semantics)."""

    def __init__(self, data: CachedDataset, start_offset: int = 0, shuffle: bool = False,
                 skip_shuffle_at_epoch_end: bool = False, shuffle_seed: int = 0, shard_rank: int = 0,
                 num_shards: int = 1, drop_shard_remainder: bool = False, repeat: bool = False) -> None:
        self.data = data
        self.start_offset = int(start_offset)
        self.shuffle = shuffle
        self.skip_shuffle_at_epoch_end = skip_shuffle_at_epoch_end
        self.shuffle_seed = shuffle_seed
        self.shard_rank = shard_rank
        self.num_shards = num_shards
        self.drop_shard_remainder = drop_shard_remainder
        self.repeat = repeat
        n = len(data)
        per = n // num_shards
        self._keys = np.arange(shard_rank, per * num_shards if drop_shard_remainder else n, num_shards)

    def __len__(self) -> int:
        return len(self._keys)

    def epoch_keys(self, epoch: int) -> np.ndarray:
        if not self.shuffle:
            return self._keys
        e = 0 if self.skip_shuffle_at_epoch_end else epoch
        return np.random.RandomState((self.shuffle_seed + e) % (2 ** 32)).permutation(self._keys)

    def __iter__(self) -> Iterator[Any]:
        n = len(self._keys)
        if n == 0:
            return
        epoch, pos = divmod(self.start_offset, n)
        info = torch.utils.data.get_worker_info()
        wid, nw = (info.id, info.num_workers) if info is not None else (0, 1)
        step = 0
        while True:
            keys = self.epoch_keys(epoch)
            for k in keys[pos:]:
                if step % nw == wid:
                    yield self.data[int(k)]
                step += 1
            if not self.repeat:
                return
            epoch, pos = epoch + 1, 0


class _CacheableDecorator:
    def __init__(self, env: Any, rank: int, size: int, training: bool, managed: bool, map_style: bool = False) -> None:
        self._env = env
        self._map_style = map_style
        self._rank, self._size = (rank, size)
        self._training = training
        self._managed = managed
        self._used = False
        self._length: Optional[int] = None
        self._offset = 0
        if training and getattr(env, "initial_workload", None) is not None:
            self._offset = int(env.initial_workload.total_batches_processed) * int(env.per_slot_batch_size)

    def is_decorator_used(self) -> bool:
        return self._used

    def get_dataset_length(self) -> int:
        if self._length is None:
            raise RuntimeError("Dataset length not yet initialized.")
        return self._length

    def _config(self) -> Dict[str, Any]:
        cfg = dict(self._env.experiment_config.get("data_layer", {}) or {})
        kind = cfg.get("type", "shared_fs")
        if kind not in SUPPORTED_TYPES:
            raise ValueError(f"data_layer type {kind!r} is not supported; supported: {list(SUPPORTED_TYPES)}")
        return cfg

    def _storage_root(self) -> pathlib.Path:
        cfg = self._config()
        if cfg.get("type", "shared_fs") == "shared_fs":
            return init_container_storage_path(cfg.get("container_storage_path"))
        return init_container_storage_path(cfg.get("local_cache_path"))

    def _object_store(self) -> Optional[Any]:
        """(client, remote prefix) for s3/gcs data layers, else None."""
        cfg = self._config()
        kind = cfg.get("type", "shared_fs")
        if kind == "shared_fs":
            return None
        from determined_1_amd.storage import rest_clients

        if kind == "s3":
            client = rest_clients.S3RestClient(cfg["bucket"], access_key=cfg.get("access_key"),
                                               secret_key=cfg.get("secret_key"), endpoint_url=cfg.get("endpoint_url"),
                                               region=cfg.get("region"))
        else:
            client = rest_clients.GCSRestClient(cfg["bucket"], endpoint_url=cfg.get("endpoint_url"),
                                                token=cfg.get("token"))
        return client, str(cfg.get("bucket_directory_path", "")).strip("/")

    @contextlib.contextmanager
    def _lock(self, path: pathlib.Path, read: bool, key: Optional[str] = None):
        """Master RW lock on ``key`` (the cache's shared identity) under a master, else an fcntl
        lock next to the local cache ``path``."""
        master = getattr(self._env, "master_addr", "")
        if self._managed and master:
            from determined_1_amd.api.rw_lock import RWLock

            with RWLock(f"{master}:{self._env.master_port}", key or str(path), read=read):
                yield
            return
        with open(str(path) + ".lock", "a+") as f:
            fcntl.flock(f, fcntl.LOCK_SH if read else fcntl.LOCK_EX)
            try:
                yield
            finally:
                fcntl.flock(f, fcntl.LOCK_UN)

    def cache_dataset(self, dataset_id: str, dataset_version: str, shuffle: bool,
                      skip_shuffle_at_epoch_end: bool) -> Callable:
        if self._training and self._used:
            raise RuntimeError("Please use both `@context.experimental.cache_train_dataset(...)` and "
                               "`@context.experimental.cache_validation_dataset(...)` exactly once.")
        self._used = True
        root = self._storage_root()
        version = dataset_version + ("_train" if self._training else "_val")
        path = root / dataset_id / version
        path.parent.mkdir(parents=True, exist_ok=True)

        store = self._object_store()
        remote = None
        if store is not None:
            client, prefix = store
            remote = "/".join(p for p in (prefix, dataset_id, version) if p)
        lock_key = f"{self._config().get('bucket', '')}/{remote}" if remote else str(path)

        def _fetch() -> bool:
            """Download a complete remote cache into ``path`` (atomically); False if none.  Called only
            under the exclusive lock; a replace that loses to a concurrent writer outside this lock's
            reach (another node's local-mode fcntl lock) still counts as a hit once meta.json is there."""
            if remote is None or not list(client.list(remote + "/meta.json")):
                return False
            tmp = pathlib.Path(tempfile.mkdtemp(prefix=".tmp_", dir=str(path.parent)))
            try:
                client.download_dir(remote, str(tmp))
                try:
                    os.replace(tmp, path)
                except OSError:
                    if not (path / "meta.json").exists():
                        raise
            finally:
                if tmp.exists():
                    shutil.rmtree(tmp, ignore_errors=True)
            logging.info(f"Downloaded cached dataset {dataset_id}:{version} from the object store.")
            return True

        def _wrap(make_dataset_fn: Callable) -> Callable:
            @functools.wraps(make_dataset_fn)
            def _decorated(*args: Any, **kwargs: Any) -> Any:
                # readers only look; every download or build happens under the exclusive lock, which
                # re-checks first, so concurrent same-node readers never race on the rename
                with self._lock(path, read=True, key=lock_key):
                    hit = (path / "meta.json").exists()
                if not hit:
                    with self._lock(path, read=False, key=lock_key):
                        if not (path / "meta.json").exists() and not _fetch():
                            stale = remove_stale_temp_dirs(path)
                            if stale:
                                logging.info(f"removed {stale} partial cache dir(s) of a killed writer")
                            logging.info(f"Caching dataset {dataset_id}:{version} to {path}.")
                            write_cache(make_dataset_fn(*args, **kwargs), path)
                            if remote is not None:
                                files = sorted(p.name for p in path.iterdir())
                                for name in [f for f in files if f != "meta.json"] + ["meta.json"]:
                                    client.upload_file(str(path / name), f"{remote}/{name}")
                if self._map_style:
                    data = CachedDataset(path)
                    if shuffle and not skip_shuffle_at_epoch_end:
                        logging.warning(
                            "cache_train/validation_dataset(shuffle=True) on a PyTorchTrial applies ONE fixed "
                            "permutation (skip_shuffle_at_epoch_end=True semantics): a map-style dataset cannot "
                            "see epoch boundaries.  Pass shuffle=True to det.pytorch.DataLoader for a per-epoch "
                            "reshuffle (docs/PARITY.md, data layer).")
                    if shuffle:
                        seed = int(getattr(self._env, "trial_seed", 0)) % (2 ** 32)
                        data.order = np.random.RandomState(seed).permutation(len(data))
                    self._length = len(data)
                    return data
                stream = CachedStream(
                    CachedDataset(path), start_offset=self._offset, shuffle=shuffle,
                    skip_shuffle_at_epoch_end=skip_shuffle_at_epoch_end, shuffle_seed=self._env.trial_seed,
                    shard_rank=self._rank, num_shards=self._size, drop_shard_remainder=self._training,
                    repeat=self._training)
                self._length = len(stream)
                return stream

            return _decorated

        return _wrap


class DataLayerContext:
    """``context.experimental`` (reference ``_data_layer/_context.py``)."""

    def __init__(self, env: Any, rank: int = 0, size: int = 1, managed: bool = False, map_style: bool = False) -> None:
        self._train = _CacheableDecorator(env, rank, size, training=True, managed=managed, map_style=map_style)
        self._val = _CacheableDecorator(env, rank, size, training=False, managed=managed, map_style=map_style)

    def cache_train_dataset(self, dataset_id: str, dataset_version: str, shuffle: bool = False,
                            skip_shuffle_at_epoch_end: bool = False) -> Callable:
        return self._train.cache_dataset(dataset_id, dataset_version, shuffle, skip_shuffle_at_epoch_end)

    def cache_validation_dataset(self, dataset_id: str, dataset_version: str, shuffle: bool = False,
                                 skip_shuffle_at_epoch_end: bool = False) -> Callable:
        return self._val.cache_dataset(dataset_id, dataset_version, shuffle, skip_shuffle_at_epoch_end)

    def get_train_cacheable(self) -> _CacheableDecorator:
        return self._train

    def get_validation_cacheable(self) -> _CacheableDecorator:
        return self._val
