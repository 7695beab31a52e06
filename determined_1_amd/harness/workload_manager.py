"""Per-workload checks, checkpoint storage and TensorBoard hooks (reference
``layers/_workload_manager.py:47-324``).

Input stream: ``(workload, args, respond)`` from the socket (or a test stream).  Output stream:
the same triples for the controller, whose raw responses (``util.wrap_metrics`` shape:
``{"metrics": ..., "stop_requested": bool}``) are checked and turned into
``{"metrics": ..., "exited_reason"?}`` for the layer above:
  * step ids must increase by one per RUN_STEP (``check_sane_workload``);
  * training batch metrics must have consistent keys;
  * the searcher metric must be present, scalar and not None/NaN in validation metrics;
  * CHECKPOINT_MODEL runs inside ``storage.store_path()`` on the chief container and answers with
    ``StorageMetadata`` (uuid, resources, framework, format);
  * ``stop_requested`` becomes ``exited_reason = USER_CANCELED``.
"""
import logging
import math
import pathlib
import tempfile
from typing import Any, Callable, Dict, Optional

import numpy as np

from determined_1_amd import errors, util, workload
from determined_1_amd.harness import timeline
from determined_1_amd.env import EnvContext, RendezvousInfo
from determined_1_amd.storage import StorageManager, StorageMetadata, list_directory


class WorkloadManager(workload.Source):
    def __init__(self, env: EnvContext, stream: workload.Stream, storage_mgr: Optional[StorageManager],
                 rendezvous_info: Optional[RendezvousInfo] = None, tensorboard_mgr: Any = None,
                 metric_writer: Any = None) -> None:
        self.env = env
        self.stream = stream
        self.storage_mgr = storage_mgr
        self.rendezvous_info = rendezvous_info
        self.tensorboard_mgr = tensorboard_mgr
        self.metric_writer = metric_writer
        self.is_chief_container = rendezvous_info is None or rendezvous_info.get_rank() == 0
        self.last_step_id = None  # type: Optional[int]

    def check_sane_workload(self, w: workload.Workload) -> None:
        if w.kind == workload.Workload.Kind.RUN_STEP and self.last_step_id is not None:
            if w.step_id != self.last_step_id + 1:
                raise errors.InternalException(
                    f"step ids must increase by one: got {w.step_id} after {self.last_step_id}")
        if w.kind == workload.Workload.Kind.RUN_STEP:
            self.last_step_id = w.step_id

    def __iter__(self) -> workload.Stream:
        for w, args, respond in self.stream:
            self.check_sane_workload(w)
            k = w.kind
            timeline.mark(f"start {k.name} step={w.step_id}")
            if k == workload.Workload.Kind.RUN_STEP:
                yield from self.yield_train_for_step(w, args, respond)
            elif k == workload.Workload.Kind.COMPUTE_VALIDATION_METRICS:
                yield from self.yield_compute_validation_metrics(w, args, respond)
            elif k == workload.Workload.Kind.CHECKPOINT_MODEL:
                yield from self.yield_checkpoint_model(w, args, respond)
            elif k == workload.Workload.Kind.TERMINATE:
                yield w, args, respond
                return
            else:
                raise AssertionError(f"unexpected workload {w}")
            timeline.mark(f"done {k.name} step={w.step_id}")

    @staticmethod
    def _exited(message: Dict[str, Any]) -> Optional[str]:
        return "USER_CANCELED" if message.get("stop_requested") else None

    def yield_train_for_step(self, w: workload.Workload, args: Any, respond: Callable) -> workload.Stream:
        def _respond(message: workload.Response) -> None:
            if isinstance(message, workload.Skipped):
                respond(message)
                return
            metrics = message["metrics"]
            util.validate_batch_metrics(metrics.get("batch_metrics", []))
            if self.metric_writer is not None:
                self.metric_writer.on_train_step_end(w.step_id, w.total_batches_processed + w.num_batches, metrics)
            if self.tensorboard_mgr is not None:
                self.tensorboard_mgr.sync()
            out = {"metrics": metrics}
            reason = self._exited(message)
            if reason:
                out["exited_reason"] = reason
            respond(out)

        yield w, args, _respond

    def yield_compute_validation_metrics(self, w: workload.Workload, args: Any, respond: Callable) -> workload.Stream:
        def _respond(message: workload.Response) -> None:
            if isinstance(message, workload.Skipped):
                respond(message)
                return
            metrics = message["metrics"]
            vm = metrics.get("validation_metrics", {})
            searcher_metric = self.env.experiment_config.get("searcher", {}).get("metric")
            if searcher_metric:
                if searcher_metric not in vm:
                    raise AssertionError(f"Search method is configured to use metric '{searcher_metric}' but model "
                                         f"definition returned validation metrics {list(vm)}.")
                v = vm[searcher_metric]
                if isinstance(v, (np.ndarray, list)) or not isinstance(v, (int, float, np.number)) or isinstance(v, bool):
                    raise AssertionError(f"searcher validation metric '{searcher_metric}' must be a scalar, got {v!r}")
                if v is None or (isinstance(v, float) and math.isnan(v)):
                    raise AssertionError(f"searcher validation metric '{searcher_metric}' is None/NaN")
            # non-JSON values (bytes) are dropped, like the reference
            metrics["validation_metrics"] = {k: x for k, x in vm.items() if not isinstance(x, (bytes, bytearray))}
            if self.metric_writer is not None:
                self.metric_writer.on_validation_step_end(w.step_id, w.total_batches_processed, metrics)
            if self.tensorboard_mgr is not None:
                self.tensorboard_mgr.sync()
            out = {"metrics": metrics}
            reason = self._exited(message)
            if reason:
                out["exited_reason"] = reason
            respond(out)

        yield w, args, _respond

    def yield_checkpoint_model(self, w: workload.Workload, args: Any, respond: Callable) -> workload.Stream:
        if not self.is_chief_container or self.storage_mgr is None:
            tmp = pathlib.Path(tempfile.mkdtemp(prefix="det-nonchief-ckpt-"))
            yield w, [tmp], lambda m: respond(workload.Skipped())
            return
        captured = {}  # type: Dict[str, Any]
        with self.storage_mgr.store_path() as (storage_id, path):
            yield w, [path], lambda m: captured.__setitem__("m", m)
            resources = list_directory(path)
        m = captured.get("m")
        if m is None or isinstance(m, workload.Skipped):
            respond(workload.Skipped() if m is not None else {"metrics": None, "exited_reason": "ERRORED"})
            return
        md = StorageMetadata(storage_id, resources, m.get("framework"), m.get("format"))
        logging.info("saved checkpoint %s (%d files)", storage_id, len(resources))
        respond({"metrics": md.__json__()})


def build_workload_manager(env: EnvContext, stream: workload.Stream, rendezvous_info: RendezvousInfo,
                           storage_mgr: StorageManager, tensorboard_mgr: Any = None,
                           metric_writer: Any = None) -> WorkloadManager:
    return WorkloadManager(env, stream, storage_mgr, rendezvous_info, tensorboard_mgr, metric_writer)
