"""Test harness helpers: fake workload streams feeding a controller directly (no master), the
same strategy as the reference's harness/tests/experiment/utils.py."""
import pathlib
from typing import Any, Dict, List, Optional, Tuple

from determined_1_amd import workload
from determined_1_amd.experimental import make_controller


def base_config(hparams: Dict[str, Any], **extra: Any) -> Dict[str, Any]:
    cfg = {"hyperparameters": dict(hparams),
           "searcher": {"name": "single", "metric": "validation_loss", "max_length": {"batches": 100}}}
    cfg.update(extra)
    return cfg


class Recorder:
    """Builds a workload stream and records every response."""

    def __init__(self) -> None:
        self.items = []  # type: List[Tuple[workload.Workload, List[Any]]]
        self.responses = []  # type: List[Any]

    def train(self, step_id: int, num_batches: int, total: int) -> "Recorder":
        self.items.append((workload.train_workload(step_id, num_batches=num_batches, total_batches_processed=total), []))
        return self

    def validate(self, step_id: int, total: int) -> "Recorder":
        self.items.append((workload.validation_workload(step_id, total_batches_processed=total), []))
        return self

    def checkpoint(self, step_id: int, total: int, path: pathlib.Path) -> "Recorder":
        self.items.append((workload.checkpoint_workload(step_id, total_batches_processed=total), [path]))
        return self

    def stream(self):
        for w, args in self.items:
            yield w, args, self.responses.append
        yield workload.terminate_workload(), [], workload.ignore_response


def run(trial_cls: Any, hparams: Dict[str, Any], rec: Recorder, load_path: Optional[pathlib.Path] = None,
        total_batches: int = 0, trial_seed: int = 0, use_gpu: bool = False, **cfg_extra: Any):
    cfg = base_config(hparams, **cfg_extra)
    init = workload.train_workload(1, num_batches=1, total_batches_processed=total_batches)
    ctrl = make_controller(trial_cls, cfg, rec.stream(), load_path=load_path, trial_seed=trial_seed,
                           initial_workload=init, use_gpu=use_gpu)
    ctrl.run()
    return ctrl, rec.responses
