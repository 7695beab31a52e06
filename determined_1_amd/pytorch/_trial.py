"""PyTorchTrial and its controller: the training hot loop.

Reference: ``harness/determined/pytorch/_pytorch_trial.py`` (controller :34-766, trial :769-1042).
Behaviour kept: workload dispatch, epoch index = batch_idx // len(loader), LR auto-stepping,
chief-only responses, batch-count-weighted validation reduction across ranks, checkpoint file
``state_dict.pth`` with ``models_state_dict / optimizers_state_dict / lr_schedulers_state_dict /
callbacks / rng_state [/ amp_state]`` plus ``code/``, legacy checkpoint paths/keys on load, and
the deprecated ``build_model()/optimizer()`` interface.

MI355X-specific changes to the loop:
  * batches arrive through ``DevicePrefetcher`` (H2D on a side stream, ``depth`` ahead);
  * per-batch training metrics stay on the GPU and are copied to the host ONCE per workload
    (the reference's per-batch ``.cpu()`` is a device sync every batch, SURVEY CS4 "hidden stall");
  * ``train_batch``/``evaluate_batch`` run under ``torch.autocast`` when AMP O1 is configured.
"""
import logging
import os
import pathlib
import random
import time
from abc import abstractmethod
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple, Union, cast

import numpy as np
import torch
import torch.nn as nn

from determined_1_amd import check, errors, trial, util, workload
from determined_1_amd.parallel import dist as pdist
from determined_1_amd.pytorch import _callback, _graph
from determined_1_amd.pytorch._context import PyTorchTrialContext
from determined_1_amd.pytorch._data import (BatchChunk, ChunkedBatches, ChunkPrefetcher, DataLoader, DevicePrefetcher,
                                            TorchData, data_length, shutdown_iterator, stacked_rows_loader)
from determined_1_amd.pytorch._lr_scheduler import LRScheduler
from determined_1_amd.pytorch._reducer import Reducer, _reduce_metrics

# (experiment) DET_COMPUTE_STREAM_HIGH_PRIO=1: run training steps on a high-priority stream
COMPUTE_STREAM_HIGH_PRIO = os.environ.get("DET_COMPUTE_STREAM_HIGH_PRIO", "0") == "1"

try:
    import cloudpickle as _pickle_module  # reference checkpoints are written with cloudpickle
except ImportError:  # pragma: no cover
    import pickle as _pickle_module  # type: ignore

CHECKPOINT_FILE = "state_dict.pth"
LEGACY_CHECKPOINT_PATHS = [["state_dict.pth"], ["determined", "state_dict.pth"], ["pedl", "state_dict.pth"],
                           ["checkpoint.pt"]]


class _HostBatches:
    """``(n, batch)`` over a host loader iterator without a device prefetch (CPU trials); ``_it``
    exposes the loader iterator to ``shutdown_iterator``."""

    def __init__(self, it: Iterator[Any], to_device: Callable[[Any], Any]) -> None:
        self._it = it
        self._to_device = to_device

    def __iter__(self) -> "_HostBatches":
        return self

    def __next__(self) -> Tuple[int, Any]:
        b = next(self._it)
        return data_length(b), self._to_device(b)


class PyTorchTrialController(trial.LoopTrialController):
    def __init__(self, trial_inst: trial.Trial, *args: Any, **kwargs: Any) -> None:
        super().__init__(*args, **kwargs)
        check.is_instance(trial_inst, PyTorchTrial, "PyTorchTrialController needs a PyTorchTrial")
        self.trial = cast(PyTorchTrial, trial_inst)
        self.context = cast(PyTorchTrialContext, self.context)
        self.callbacks = self.trial.build_callbacks()
        self._apply_backwards_compatibility()
        check.gt_eq(len(self.context.models), 1,
                    "Must have at least one model. This might be caused by not wrapping your model with wrap_model()")
        check.gt_eq(len(self.context.optimizers), 1,
                    "Must have at least one optimizer. This might be caused by not wrapping your optimizer with "
                    "wrap_optimizer()")
        self._check_evaluate_implementation()
        self.validation_loader = None  # type: Optional[torch.utils.data.DataLoader]
        self._set_data_loaders()
        self.training_iterator = self._make_train_iterator()
        self._graph = None  # type: Optional[_graph.TrainStepGraph]
        self._graph_checked = False
        self._hp_stream = None  # type: Any  # COMPUTE_STREAM_HIGH_PRIO
        self._eval_graph = None  # type: Optional[_graph.EvalStepGraph]
        # arenas / fused optimizers / bucketers, then restore, then rank-0 broadcast
        self.context._finalize()
        self._load()
        if self.dist_config.use and pdist.is_initialized():
            self.context._broadcast_state()

    # ------------------------------------------------------------------------------------------
    @staticmethod
    def pre_execute_hook(env: Any, dist_config: Any) -> None:
        if dist_config.use:
            device = pdist.local_cuda_device(int(pdist.RankInfo.from_env().local_rank)) \
                if torch.cuda.is_available() else torch.device("cpu")
            if device.type == "cuda":
                torch.cuda.set_device(device)
                from determined_1_amd.parallel.ddp import apply_rccl_env

                apply_rccl_env({"rccl": getattr(dist_config, "rccl", {})})
            pdist.init_process_groups(device)
        PyTorchTrialController._set_random_seeds(env.trial_seed)
        # One process drives one GPU here, so autograd's per-device worker thread only adds a
        # cross-thread handoff per backward (measured +8-13% BERT-base throughput without it,
        # round-1 A/B, profiles/r1_bench_bert_base_bs12.json).  DET_AUTOGRAD_THREADS=1 restores the stock engine.
        if os.environ.get("DET_AUTOGRAD_THREADS", "0") != "1":
            torch.autograd.set_multithreading_enabled(False)

    @staticmethod
    def _set_random_seeds(seed: int) -> None:
        random.seed(seed)
        np.random.seed(seed)
        torch.random.manual_seed(seed)
        from determined_1_amd.ops import transformer as _tf

        _tf.reset_rng()  # the native dropout stream follows the new torch seed

    @staticmethod
    def from_trial(*args: Any, **kwargs: Any) -> trial.TrialController:
        return PyTorchTrialController(*args, **kwargs)

    @staticmethod
    def from_native(*args: Any, **kwargs: Any) -> trial.TrialController:
        raise NotImplementedError("PyTorchTrial only supports the Trial API")

    @staticmethod
    def supports_mixed_precision() -> bool:
        return True

    @staticmethod
    def supports_averaging_training_metrics() -> bool:
        return True

    # ------------------------------------------------------------------------------------------
    def _check_evaluate_implementation(self) -> None:
        check.not_eq(
            self._evaluate_batch_defined(),
            self._evaluate_full_dataset_defined(),
            "Please define exactly one of: `evaluate_batch()` or `evaluate_full_dataset()`. For most use cases "
            "`evaluate_batch()` is recommended because it can be parallelized across all devices.",
        )

    def _evaluate_batch_defined(self) -> bool:
        return util.is_overridden(self.trial.evaluate_batch, PyTorchTrial)

    def _evaluate_full_dataset_defined(self) -> bool:
        return util.is_overridden(self.trial.evaluate_full_dataset, PyTorchTrial)

    def _apply_backwards_compatibility(self) -> None:
        t = self.trial
        legacy = (util.is_overridden(t.build_model, PyTorchTrial) or util.is_overridden(t.optimizer, PyTorchTrial)
                  or util.is_overridden(t.create_lr_scheduler, PyTorchTrial))
        if not legacy:
            return
        logging.warning("build_model(), optimizer(), and create_lr_scheduler() are deprecated; wrap models and "
                        "optimizers in __init__ and call context.backward()/context.step_optimizer().")
        check.true(util.is_overridden(t.build_model, PyTorchTrial) and util.is_overridden(t.optimizer, PyTorchTrial),
                   "Both build_model() and optimizer() must be defined if any of build_model(), optimizer(), and "
                   "create_lr_scheduler() are defined.")
        model = self.context.wrap_model(t.build_model())
        optim = self.context.wrap_optimizer(t.optimizer(model))
        lr_scheduler = t.create_lr_scheduler(optim)
        if lr_scheduler is not None:
            opt = getattr(lr_scheduler._scheduler, "optimizer", None)
            if opt is not None:
                check.is_in(opt, self.context.optimizers, "Must use a wrapped optimizer in create_lr_scheduler")
            self.context.lr_schedulers.append(lr_scheduler)
        if self.env.experiment_config.mixed_precision_enabled():
            self.context.configure_apex_amp(
                models=model, optimizers=optim,
                opt_level=self.env.experiment_config.get("optimizations", {}).get("mixed_precision", "O0"))
        train_batch = cast(Callable, t.train_batch)

        def new_train_batch(batch: TorchData, epoch_idx: int, batch_idx: int) -> Any:
            tr_metrics = train_batch(batch=batch, model=model, epoch_idx=epoch_idx, batch_idx=batch_idx)
            if isinstance(tr_metrics, torch.Tensor):
                tr_metrics = {"loss": tr_metrics}
            check.is_instance(tr_metrics, dict, "train_batch() must return a dictionary mapping string names to "
                                                "Tensor metrics")
            check.is_in("loss", tr_metrics.keys(), 'Please include "loss" in your training metrics.')

            def clip_grads(parameters: Iterator) -> None:
                for cb in self.callbacks.values():
                    cb.on_before_optimizer_step(parameters)

            self.context.backward(tr_metrics["loss"])
            self.context.step_optimizer(self.context.optimizers[0], clip_grads=clip_grads)
            return tr_metrics

        t.__setattr__("train_batch", new_train_batch)
        if self._evaluate_batch_defined():
            evaluate_batch = cast(Callable, t.evaluate_batch)
            t.__setattr__("evaluate_batch", lambda batch: evaluate_batch(model=model, batch=batch))
        if self._evaluate_full_dataset_defined():
            efd = cast(Callable, t.evaluate_full_dataset)
            t.__setattr__("evaluate_full_dataset", lambda data_loader: efd(model=model, data_loader=data_loader))

    def _set_data_loaders(self) -> None:
        skip = self.env.initial_workload.total_batches_processed
        nreplicas = self.context.distributed.get_size()
        rank = self.context.distributed.get_rank()
        self.training_loader = self.trial.build_training_data_loader().get_data_loader(
            repeat=True, skip=skip, num_replicas=nreplicas, rank=rank)
        self.context._epoch_len = len(self.training_loader)
        vds = self.trial.build_validation_data_loader()
        if self._evaluate_batch_defined():
            self.validation_loader = vds.get_data_loader(repeat=False, skip=0, num_replicas=nreplicas, rank=rank)
        elif self.is_chief:
            self.validation_loader = vds.get_data_loader(repeat=False, skip=0, num_replicas=1, rank=0)

    def _make_train_iterator(self) -> Iterator[Any]:
        """Per-batch ``(n, device_batch)`` iterator, or -- with ``optimizations.hip_graph_batches``
        K > 1 and a stacked-rows loader -- an iterator of device ``BatchChunk``s of up to K batches
        (one dataset call and one H2D copy per leaf per chunk; chunks never cross an epoch)."""
        dev = self.context.device
        self._pending = None  # type: Optional[BatchChunk]  # rest of a chunk split at a step end
        self._chunked = self._graph_batches() > 1 and stacked_rows_loader(self.training_loader)
        if self._chunked:
            unit = int(self.env.experiment_config.get("scheduling_unit", 100) or 100)
            chunks = ChunkedBatches(self.training_loader, self._graph_batches(), epoch_len=len(self.training_loader),
                                    start=self.env.initial_workload.total_batches_processed, unit=unit)
            return ChunkPrefetcher(chunks, dev, depth=2)
        it = iter(self.training_loader)
        if dev.type == "cuda":
            return DevicePrefetcher(it, dev, depth=2)

        return _HostBatches(it, self.context.to_device)

    def _graph_batches(self) -> int:
        env = os.environ.get("DET_GRAPH_BATCHES")
        if env:
            return max(1, int(env))
        opt = self.env.experiment_config.get("optimizations", {}) or {}
        return max(1, int(opt.get("hip_graph_batches", 1) or 1))

    def _chunk_graph_ok(self) -> bool:
        """K steps in one replay apply one set of hyper-parameters: no per-batch LR schedules."""
        return self._graph is not None and all(
            s._step_mode == LRScheduler.StepMode.STEP_EVERY_EPOCH for s in self.context.lr_schedulers)

    # ------------------------------------------------------------------------------------------
    def run(self) -> None:
        try:
            self._run()
        finally:
            shutdown_iterator(self.training_iterator)

    def _run(self) -> None:
        for w, args, respond in self.workloads:
            if w.kind == workload.Workload.Kind.RUN_STEP:
                respond(util.wrap_metrics(self._train_for_step(w.step_id, w.num_batches, w.total_batches_processed),
                                          self.context.get_stop_requested()))
            elif w.kind == workload.Workload.Kind.COMPUTE_VALIDATION_METRICS:
                respond(util.wrap_metrics(self._compute_validation_metrics(), self.context.get_stop_requested()))
            elif w.kind == workload.Workload.Kind.CHECKPOINT_MODEL:
                check.len_eq(args, 1)
                check.is_instance(args[0], pathlib.Path)
                respond(self._save(cast(pathlib.Path, args[0])))
            elif w.kind == workload.Workload.Kind.TERMINATE:
                respond({} if self.is_chief else workload.Skipped())
                break
            else:
                raise AssertionError(f"Unexpected workload: {w.kind}")

    def _hip_graph_enabled(self) -> bool:
        env = os.environ.get("DET_HIP_GRAPH")
        if env is not None:
            return env not in ("", "0")
        opt = self.env.experiment_config.get("optimizations", {}) or {}
        return bool(opt.get("hip_graph", False))

    def get_epoch_idx(self, batch_id: int) -> int:
        return batch_id // len(self.training_loader)

    def _auto_step_lr_scheduler_per_batch(self, batch_idx: int, lr_scheduler: LRScheduler) -> None:
        if lr_scheduler._step_mode == LRScheduler.StepMode.STEP_EVERY_BATCH:
            lr_scheduler.step()
        elif lr_scheduler._step_mode == LRScheduler.StepMode.STEP_EVERY_EPOCH:
            mod = (batch_idx + 1) % len(self.training_loader)
            if mod == 0 or mod < self.dist_config.aggregation_frequency:
                lr_scheduler.step()

    def _train_for_step(self, step_id: int, num_batches: int, total_batches_processed: int) -> workload.Response:
        if not (COMPUTE_STREAM_HIGH_PRIO and self.context.device.type == "cuda"):
            return self._train_for_step_on_stream(step_id, num_batches, total_batches_processed)
        # the training step on a high-priority stream: work forked to a side stream (the conv weight
        # gradients, ops/arena.py side_work) then yields the CUs to the input-gradient chain, which
        # is the step's critical path
        dev = self.context.device
        if self._hp_stream is None:
            self._hp_stream = torch.cuda.Stream(dev, priority=-1)
        default = torch.cuda.current_stream(dev)
        self._hp_stream.wait_stream(default)
        try:
            with torch.cuda.stream(self._hp_stream):
                return self._train_for_step_on_stream(step_id, num_batches, total_batches_processed)
        finally:
            default.wait_stream(self._hp_stream)

    def _train_for_step_on_stream(self, step_id: int, num_batches: int, total_batches_processed: int) -> workload.Response:
        check.gt(step_id, 0)
        for model in self.context.models:
            model.train()
        start, end = total_batches_processed, total_batches_processed + num_batches
        per_batch = []  # type: List[Dict[str, Any]]
        num_inputs = 0
        timers = self.context._timers
        batch_idx = start
        while batch_idx < end:
            t_data = time.perf_counter()
            if not self._chunked:
                n, batch = next(self.training_iterator)
                num_inputs += n
                per_batch.append(self._train_one(batch, batch_idx, time.perf_counter() - t_data))
                batch_idx += 1
                continue
            chunk = self._pending if self._pending is not None else next(self.training_iterator)
            self._pending = None
            if batch_idx + len(chunk) > end:  # the step ends inside this chunk: the rest opens the next step
                chunk, self._pending = chunk.split(end - batch_idx)
            k = len(chunk)
            num_inputs += sum(chunk.sizes)
            if self._chunk_graph_ok():
                assert self._graph is not None
                timers.batch_start(time.perf_counter() - t_data)
                self.context._current_batch_idx = batch_idx
                self.context._loss_ids = {}
                stacked = self._graph.run_chunk(chunk, self.get_epoch_idx(batch_idx), batch_idx,
                                                capture=k == self._graph_batches())
                if stacked is not None:
                    per_batch.append(_StackedMetrics(stacked, k))
                else:
                    per_batch.extend(_detach_metrics(m) for m in self._graph.last_chunk_metrics or [])
                for i in range(k):
                    for lr_scheduler in self.context.lr_schedulers:
                        self._auto_step_lr_scheduler_per_batch(batch_idx + i, lr_scheduler)
            else:  # no multi-batch graph (CPU, ineligible, first batch): the chunk's batches one by one
                for i, b in enumerate(chunk.batches):
                    per_batch.append(self._train_one(b, batch_idx + i, time.perf_counter() - t_data))
                    t_data = time.perf_counter()
            batch_idx += k
        per_batch = _batch_metrics_to_host(per_batch)
        self.last_step_timers = timers.report(step_id)
        if self.dist_config.use and self.dist_config.average_training_metrics:
            per_batch = self._average_training_metrics(per_batch)
        if self.dist_config.use:
            num_inputs *= self.context.distributed.get_size()
        metrics = util.make_metrics(num_inputs, per_batch)
        if not self.is_chief:
            return workload.Skipped()
        logging.debug(f"Done training step: {num_inputs} records in {num_batches} batches.")
        return metrics

    def _train_one(self, batch: Any, batch_idx: int, data_seconds: float) -> Dict[str, Any]:
        self.context._timers.batch_start(data_seconds)
        self.context._current_batch_idx = batch_idx
        self.context._loss_ids = {}
        if self._graph is not None:
            tr_metrics = self._graph.run(batch, self.get_epoch_idx(batch_idx), batch_idx)
        else:
            with self.context._autocast():
                tr_metrics = self.trial.train_batch(batch=batch, epoch_idx=self.get_epoch_idx(batch_idx),
                                                    batch_idx=batch_idx)
            if not self._graph_checked and self.context._finalized:
                self._graph_checked = True
                self._graph, _ = _graph.build(self.context, self.trial.train_batch, self._hip_graph_enabled())
        for lr_scheduler in self.context.lr_schedulers:
            self._auto_step_lr_scheduler_per_batch(batch_idx, lr_scheduler)
        # detached copies only: a live autograd graph keeps its AccumulateGrad nodes bound to this
        # stream, which breaks a hipGraph capture of the next batch
        return _detach_metrics(tr_metrics)

    def _average_training_metrics(self, per_batch_metrics: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
        gathered = pdist.gather_to_chief(per_batch_metrics)
        if not self.is_chief:
            return per_batch_metrics
        assert gathered is not None
        out = []
        for bi in range(len(per_batch_metrics)):
            row = {}
            for name, v0 in per_batch_metrics[bi].items():
                vals = [g[bi][name] for g in gathered if g[bi][name] is not None]
                try:
                    avg = np.mean(np.array(vals, dtype=np.float64), axis=0)
                    row[name] = np.array(avg) if isinstance(v0, np.ndarray) else avg
                except (TypeError, ValueError):
                    row[name] = v0
            out.append(row)
        return out

    # ------------------------------------------------------------------------------------------
    @torch.no_grad()
    def _compute_validation_metrics(self) -> workload.Response:
        for model in self.context.models:
            model.eval()
        for cb in self.callbacks.values():
            if util.is_overridden(cb.on_validation_step_start, _callback.PyTorchCallback):
                logging.warning("on_validation_step_start is deprecated, please use on_validation_start instead")
            cb.on_validation_step_start()
        for cb in self.callbacks.values():
            cb.on_validation_start()
        num_inputs = 0
        metrics = {}  # type: Optional[Dict[str, Any]]
        if self._evaluate_batch_defined():
            keys = None
            batch_metrics = []
            loader = cast(torch.utils.data.DataLoader, self.validation_loader)
            check.gt(len(loader), 0)
            if self._eval_graph is None and self._hip_graph_enabled() and self.context.device.type == "cuda":
                self._eval_graph = _graph.EvalStepGraph(self.context, self.trial.evaluate_batch)
            for vm in self._validation_batches(loader):
                if isinstance(vm, _StackedMetrics):  # K batches of one multi-batch replay
                    names = vm.stacked.keys()
                else:
                    check.is_instance(vm, dict, "evaluate_batch() must return a dictionary of string names to "
                                                "Tensor metrics")
                    names = vm.keys()
                if keys is None:
                    keys = names
                else:
                    check.eq(keys, names, "Validation metric names must match across all batches of data.")
                if isinstance(vm, _StackedMetrics):
                    batch_metrics.append(vm)
                else:
                    batch_metrics.append({k: (v.detach().float() if isinstance(v, torch.Tensor) else v)
                                          for k, v in vm.items()})
            num_inputs += self._val_inputs
            batch_metrics = _batch_metrics_to_host(batch_metrics)
            metrics = self._reduce_metrics(batch_metrics, keys, self._prepare_metrics_reducers(keys))
            if self.dist_config.use:
                num_inputs *= self.context.distributed.get_size()
        else:
            check.true(self._evaluate_full_dataset_defined())
            if self.is_chief:
                loader = cast(torch.utils.data.DataLoader, self.validation_loader)
                metrics = self.trial.evaluate_full_dataset(data_loader=loader)
                check.is_instance(metrics, dict, f"eval() must return a dictionary, got {type(metrics)}.")
                metrics = _convert_metrics_to_numpy(cast(Dict[str, Any], metrics))
                num_inputs = self.context.get_per_slot_batch_size() * len(loader)
        if self.dist_config.use and any(
            util.is_overridden(c.on_validation_end, _callback.PyTorchCallback)
            or util.is_overridden(c.on_validation_step_end, _callback.PyTorchCallback)
            for c in self.callbacks.values()
        ):
            metrics = pdist.broadcast_object(metrics, src=0)
        for cb in self.callbacks.values():
            cb.on_validation_step_end(cast(Dict[str, Any], metrics))
        for cb in self.callbacks.values():
            cb.on_validation_end(cast(Dict[str, Any], metrics))
        if not self.is_chief:
            return workload.Skipped()
        return {"num_inputs": num_inputs, "validation_metrics": metrics}

    def _validation_batches(self, loader: Any) -> Iterator[Any]:
        """evaluate_batch metrics per validation batch; K batches per dataset call / H2D copy /
        hipGraph replay when ``hip_graph_batches`` > 1 and the loader yields stacked rows."""
        self._val_inputs = 0
        k = self._graph_batches()
        if k > 1 and stacked_rows_loader(loader):
            for chunk in ChunkedBatches(loader, k):
                self._val_inputs += sum(chunk.sizes)
                dev = BatchChunk(self.context.to_device(chunk.stacked), chunk.sizes)
                if self._eval_graph is not None:
                    stacked = self._eval_graph.run_chunk(dev)
                    if stacked is not None:
                        yield _StackedMetrics(stacked, len(chunk))
                    else:
                        yield from self._eval_graph.last_chunk_metrics or []
                else:
                    for b in dev.batches:
                        with self.context._autocast():
                            yield self.trial.evaluate_batch(batch=b)
            return
        for batch in loader:
            self._val_inputs += data_length(batch)
            batch = self.context.to_device(batch)
            if self._eval_graph is not None:
                yield self._eval_graph.run(batch)
            else:
                with self.context._autocast():
                    yield self.trial.evaluate_batch(batch=batch)

    def _prepare_metrics_reducers(self, keys: Any) -> Dict[str, Reducer]:
        red = self.trial.evaluation_reducer()
        out = {}  # type: Dict[str, Reducer]
        if isinstance(red, dict):
            check.eq(set(red.keys()), set(keys),
                     "Please provide a single evaluation reducer or provide a reducer for every validation metric. "
                     f"Expected keys: {keys}, provided keys: {red.keys()}.")
            out = dict(red)
        elif isinstance(red, Reducer):
            out = {k: red for k in keys}
        for k in keys:
            check.true(isinstance(out.get(k), Reducer),
                       "Please select `determined.pytorch.Reducer` for reducing validation metrics.")
        return out

    def _reduce_metrics(self, batch_metrics: List[Dict[str, Any]], keys: Any,
                        reducers: Dict[str, Reducer]) -> Optional[Dict[str, Any]]:
        metrics = {name: _reduce_metrics(reducers[name], np.stack([b[name] for b in batch_metrics], axis=0), None)
                   for name in keys or []}
        if self.dist_config.use and pdist.is_initialized():
            loader = cast(torch.utils.data.DataLoader, self.validation_loader)
            gathered = pdist.gather_to_chief((metrics, len(loader)))
            if not self.is_chief:
                return {}
            assert gathered is not None
            per_proc = [g[1] for g in gathered]
            metrics = {name: _reduce_metrics(reducers[name], np.stack([np.asarray(g[0][name]) for g in gathered], axis=0),
                                             per_proc)
                       for name in keys or []}
        return metrics

    # ------------------------------------------------------------------------------------------
    def _load(self) -> None:
        if not self.load_path:
            return
        checkpoint = None
        for parts in LEGACY_CHECKPOINT_PATHS:
            p = self.load_path.joinpath(*parts)
            if p.exists():
                checkpoint = torch.load(str(p), map_location="cpu", weights_only=False)
                break
        if checkpoint is None:
            raise errors.CheckpointNotFoundException(f"no checkpoint file found under {self.load_path}")
        ctx = self.context
        if "model_state_dict" in checkpoint:
            check.not_in("models_state_dict", checkpoint)
            check.eq(len(ctx.models), 1)
            ctx.models[0].load_state_dict(checkpoint["model_state_dict"])
        else:
            for idx, model in enumerate(ctx.models):
                model.load_state_dict(checkpoint["models_state_dict"][idx])
        ctx._sync_master_weights()
        if "optimizer_state_dict" in checkpoint:
            check.not_in("optimizers_state_dict", checkpoint)
            check.eq(len(ctx.optimizers), 1)
            ctx.optimizers[0].load_state_dict(checkpoint["optimizer_state_dict"])
        else:
            for idx, opt in enumerate(ctx.optimizers):
                opt.load_state_dict(checkpoint["optimizers_state_dict"][idx])
        if "lr_scheduler" in checkpoint:
            check.not_in("lr_schedulers_state_dict", checkpoint)
            check.eq(len(ctx.lr_schedulers), 1)
            ctx.lr_schedulers[0].load_state_dict(checkpoint["lr_scheduler"])
        else:
            for idx, sched in enumerate(ctx.lr_schedulers):
                sched.load_state_dict(checkpoint["lr_schedulers_state_dict"][idx])
        if "amp_state" in checkpoint:
            if ctx._amp is not None:
                ctx._amp.load_state_dict(checkpoint["amp_state"])
            else:
                logging.warning("There exists amp_state in checkpoint but the experiment is not using AMP.")
        elif ctx._amp is not None:
            logging.warning("The experiment is using AMP but amp_state does not exist in the checkpoint.")
        if "rng_state" in checkpoint:
            rs = checkpoint["rng_state"]
            np.random.set_state(rs["np_rng_state"])
            random.setstate(rs["random_rng_state"])
            torch.random.set_rng_state(rs["cpu_rng_state"])
            if torch.cuda.is_available() and ctx.device.type == "cuda":
                if "gpu_rng_state" in rs:
                    torch.cuda.set_rng_state(rs["gpu_rng_state"], device=ctx.device)
                else:
                    logging.warning("The system has a gpu but no gpu_rng_state exists in the checkpoint.")
            elif "gpu_rng_state" in rs:
                logging.warning("There exists gpu_rng_state in checkpoint but the system has no gpu.")
            if "det_dropout_rng" in rs:
                from determined_1_amd.ops import transformer as _tf

                _tf.set_rng_state(rs["det_dropout_rng"])
        else:
            logging.warning("The checkpoint has no random state to restore.")
        if checkpoint.get("accumulated_grads") is not None and self.is_chief:
            # the chief holds the ranks' summed partial window (see _partial_window_grads); the other
            # ranks continue the window from zero
            ctx._restored_grads = checkpoint["accumulated_grads"]
        cb_state = checkpoint.get("callbacks", {})
        for name, cb in self.callbacks.items():
            if name in cb_state:
                cb.load_state_dict(cb_state[name])
            elif util.is_overridden(cb.load_state_dict, _callback.PyTorchCallback):
                logging.warning(f"Callback '{name}' implements load_state_dict(), but no callback state was found "
                                "for that name when restoring from checkpoint.")

    def _save(self, path: pathlib.Path) -> workload.Response:
        partial = self.context._partial_window_grads()  # a collective across ranks: before the chief check
        if not self.is_chief:
            return workload.Skipped()
        path.mkdir(parents=True, exist_ok=True)
        util.write_user_code(path)
        ctx = self.context
        rng_state = {
            "cpu_rng_state": torch.random.get_rng_state(),
            "np_rng_state": np.random.get_state(),
            "random_rng_state": random.getstate(),
        }
        if torch.cuda.is_available() and ctx.device.type == "cuda":
            rng_state["gpu_rng_state"] = torch.cuda.get_rng_state(ctx.device)
        from determined_1_amd.ops import transformer as _tf

        rng_state["det_dropout_rng"] = _tf.rng_state()
        ckpt = {
            "models_state_dict": [m.state_dict() for m in ctx.models],
            "optimizers_state_dict": [o.state_dict() for o in ctx.optimizers],
            "lr_schedulers_state_dict": [s.state_dict() for s in ctx.lr_schedulers],
            "callbacks": {name: cb.state_dict() for name, cb in self.callbacks.items()},
            "rng_state": rng_state,
        }
        if ctx._amp is not None:
            ckpt["amp_state"] = ctx._amp_state_dict()
        if partial is not None:
            ckpt["accumulated_grads"] = partial
        torch.save(ckpt, str(path.joinpath(CHECKPOINT_FILE)), pickle_module=_pickle_module)
        for cb in self.callbacks.values():
            cb.on_checkpoint_end(str(path))
        return {"framework": f"torch-{torch.__version__}", "format": "cloudpickle"}


class _StackedMetrics:
    """Metrics of K batches from one multi-batch replay: {name: [K] tensor}."""

    def __init__(self, stacked: Dict[str, torch.Tensor], k: int) -> None:
        self.stacked = stacked
        self.k = k


def _detach_metrics(tr_metrics: Any) -> Dict[str, Any]:
    if isinstance(tr_metrics, torch.Tensor):
        tr_metrics = {"loss": tr_metrics}
    check.is_instance(tr_metrics, dict, "train_batch() must return a dictionary mapping string names to "
                                        f"Tensor metrics, got {type(tr_metrics)}")
    return {k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in tr_metrics.items()}


def _expand_stacked(per_batch: List[Any]) -> List[Dict[str, Any]]:
    """Per-batch metric dicts, multi-batch entries split into 0-d views (no device work)."""
    out = []  # type: List[Dict[str, Any]]
    for m in per_batch:
        if isinstance(m, _StackedMetrics):
            out.extend({k: v[i] for k, v in m.stacked.items()} for i in range(m.k))
        else:
            out.append(m)
    return out


def _batch_metrics_to_host(entries: List[Any]) -> List[Dict[str, Any]]:
    """Per-batch metric dicts (numpy) of a step or validation pass whose entries are per-batch dicts
    and/or ``_StackedMetrics`` of multi-batch replays.  When every entry is stacked (the chunked
    hipGraph path), each metric is concatenated on the device and all of them come back in one copy,
    without a 0-d view, detach and dict per batch first (~5 us a batch of host time: ~1,600 RUN_STEP
    and validation batches per ASHA container epoch)."""
    if entries and all(isinstance(e, _StackedMetrics) for e in entries):
        keys = list(entries[0].stacked.keys())
        if keys and all(list(e.stacked.keys()) == keys for e in entries) and all(
                isinstance(v, torch.Tensor) and v.dim() == 1 for e in entries for v in e.stacked.values()):
            cols = [torch.cat([e.stacked[k] for e in entries]).float() for k in keys]
            host = torch.stack(cols).cpu().numpy()  # [keys, batches]
            return [dict(zip(keys, row)) for row in host.T]
    return _metrics_to_host(_expand_stacked(entries))


def _metrics_to_host(batch_metrics: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
    """Convert per-batch tensor metrics to numpy with ONE device->host copy per device."""
    if not batch_metrics:
        return batch_metrics
    flat = []  # type: List[torch.Tensor]
    where = []  # type: List[Tuple[int, str]]
    for i, m in enumerate(batch_metrics):
        for k, v in m.items():
            if isinstance(v, torch.Tensor):
                # numpy has no bfloat16: widen low-precision metrics (O2 models) on device
                flat.append(v.detach().float() if v.dtype in (torch.bfloat16, torch.float16) else v.detach())
                where.append((i, k))
    if not flat:
        return batch_metrics
    out = [dict(m) for m in batch_metrics]
    by_dev = {}  # type: Dict[Any, List[int]]
    for j, t in enumerate(flat):
        by_dev.setdefault((t.device, t.dtype, t.dim() == 0), []).append(j)
    for (dev, _dt, scalar), idxs in by_dev.items():
        if scalar and len(idxs) > 1:
            host = torch.stack([flat[j] for j in idxs]).cpu().numpy()
            for r, j in enumerate(idxs):
                i, k = where[j]
                out[i][k] = host[r]
        else:
            for j in idxs:
                i, k = where[j]
                out[i][k] = flat[j].cpu().numpy()
    return out


def _convert_metrics_to_numpy(metrics: Dict[str, Any]) -> Dict[str, Any]:
    for k, v in metrics.items():
        if isinstance(v, torch.Tensor):
            v = v.detach()
            metrics[k] = (v.float() if v.dtype in (torch.bfloat16, torch.float16) else v).cpu().numpy()
    return metrics


class PyTorchTrial(trial.Trial):
    """Subclass this to define a PyTorch trial: build models/optimizers/schedulers in
    ``__init__`` (wrapped through ``context``), implement ``train_batch``, the data loaders, and
    exactly one of ``evaluate_batch`` / ``evaluate_full_dataset``."""

    trial_controller_class = PyTorchTrialController
    trial_context_class = PyTorchTrialContext

    @abstractmethod
    def __init__(self, context: PyTorchTrialContext) -> None:
        pass

    def build_model(self) -> nn.Module:  # deprecated interface
        pass  # type: ignore

    def optimizer(self, model: nn.Module) -> torch.optim.Optimizer:  # deprecated interface
        pass  # type: ignore

    def create_lr_scheduler(self, optimizer: torch.optim.Optimizer) -> Optional[LRScheduler]:  # deprecated
        pass

    @abstractmethod
    def train_batch(self, batch: TorchData, epoch_idx: int, batch_idx: int) -> Union[torch.Tensor, Dict[str, Any]]:
        pass

    @abstractmethod
    def build_training_data_loader(self) -> DataLoader:
        pass

    @abstractmethod
    def build_validation_data_loader(self) -> DataLoader:
        pass

    def build_callbacks(self) -> Dict[str, _callback.PyTorchCallback]:
        return {}

    def evaluate_batch(self, batch: TorchData) -> Dict[str, Any]:
        pass  # type: ignore

    def evaluation_reducer(self) -> Union[Reducer, Dict[str, Reducer]]:
        return Reducer.AVG

    def evaluate_full_dataset(self, data_loader: torch.utils.data.DataLoader) -> Dict[str, Any]:
        pass  # type: ignore


def reset_parameters(model: torch.nn.Module) -> None:
    """Deprecated reference helper (``harness/determined/pytorch/_pytorch_trial.py:1023``): call
    ``reset_parameters()`` on every submodule that defines it."""
    logging.warning("det.pytorch.reset_parameters() is deprecated; modules should reset themselves in __init__().")
    for m in model.modules():
        fn = getattr(m, "reset_parameters", None)
        if callable(fn):
            fn()
