"""Metric writers and event-file sync to checkpoint storage."""
import os
import shutil
import tempfile
from typing import Any, Dict, Optional

from determined_1_amd.tensorboard.events import EventFileWriter


def get_base_path(checkpoint_storage: Dict[str, Any], experiment_id: str, trial_id: str) -> str:
    host = checkpoint_storage.get("host_path", "/tmp")
    sp = checkpoint_storage.get("storage_path")
    root = os.path.join(host, sp) if sp and not os.path.isabs(sp) else (sp or host)
    return os.path.join(root, "tensorboard", "experiment", str(experiment_id), "trial", str(trial_id))


class TensorboardManager:
    """Copies new/changed event files from ``base_dir`` to the storage path."""

    def __init__(self, base_dir: str, sync_path: Optional[str]) -> None:
        self.base_dir = base_dir
        self.sync_path = sync_path
        self._synced = {}  # type: Dict[str, float]
        os.makedirs(base_dir, exist_ok=True)

    def sync(self) -> None:
        if not self.sync_path:
            return
        for root, _, files in os.walk(self.base_dir):
            for f in files:
                if "tfevents" not in f:
                    continue
                p = os.path.join(root, f)
                m = os.path.getmtime(p)
                if self._synced.get(p) == m:
                    continue
                dst = os.path.join(self.sync_path, os.path.relpath(p, self.base_dir))
                os.makedirs(os.path.dirname(dst), exist_ok=True)
                shutil.copyfile(p, dst)
                self._synced[p] = m


class MetricWriter:
    """``Determined/<name>`` per batch and ``val_<name>`` per validation (scalars only)."""

    def __init__(self, logdir: str) -> None:
        self.writer = EventFileWriter(logdir)

    @staticmethod
    def _scalar(v: Any) -> Optional[float]:
        try:
            f = float(v)
        except (TypeError, ValueError):
            return None
        return f

    def on_train_step_end(self, step_id: int, total_batches: int, metrics: Dict[str, Any]) -> None:
        bm = metrics.get("batch_metrics") or []
        first = total_batches - len(bm)
        for i, m in enumerate(bm):
            for k, v in m.items():
                f = self._scalar(v)
                if f is not None:
                    self.writer.add_scalar(f"Determined/{k}", f, first + i + 1)
        self.writer.flush()

    def on_validation_step_end(self, step_id: int, total_batches: int, metrics: Dict[str, Any]) -> None:
        for k, v in (metrics.get("validation_metrics") or {}).items():
            f = self._scalar(v)
            if f is not None:
                self.writer.add_scalar(k if k.startswith("val") else f"val_{k}", f, total_batches)
        self.writer.flush()


def build(env: Any, checkpoint_storage: Dict[str, Any]) -> TensorboardManager:
    # per host account: trial processes of different users (agent user groups) share the host's /tmp
    base = os.path.join(tempfile.gettempdir(), f"tensorboard-{os.getuid()}",
                        f"{env.det_experiment_id}-{env.det_trial_id}-{os.getpid()}")
    sync = None
    if checkpoint_storage.get("type", "shared_fs") == "shared_fs":
        sync = get_base_path(checkpoint_storage, env.det_experiment_id, env.det_trial_id)
    return TensorboardManager(base, sync)
