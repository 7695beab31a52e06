"""No-op trial for control-plane tests (mirrors the reference e2e fixture
``e2e_tests/tests/fixtures/no_op/model_def.py:17-172``): no real training, synthetic decreasing
metrics, checkpoints are a small JSON file, optional chaos (random failures) to exercise restarts.

Hyperparameters: ``metrics_base`` (0.9), ``metrics_progression`` (decreasing|increasing|constant),
``chaos_probability{,_train,_validate,_checkpoint}``, ``fail_on_first_validation``,
``fail_on_checkpoint_save``, ``validation_set_size`` (num_inputs), ``sleep`` (s per step),
``invalid_hp`` (raise InvalidHP at construction), ``log_lines`` / ``log_seconds`` (print that
many stdout lines per step, spread over that many seconds: log-shipping load tests).
"""
import json
import os
import pathlib
import random
import time
from typing import Any, Dict

from determined_1_amd import errors, trial


class NoOpTrialController(trial.CallbackTrialController):
    CHECKPOINT_FILENAME = "no_op_checkpoint"

    def __init__(self, *args: Any, **kwargs: Any) -> None:
        self.metric = 0.0
        self.trained_steps = 0
        super().__init__(*args, **kwargs)
        hp = self.context.get_hparams()
        if hp.get("invalid_hp"):
            raise errors.InvalidHP("invalid hyperparameter configuration")
        self.metric = float(hp.get("metrics_base", 0.9)) if self.load_path is None else self.metric
        self.chaos = random.Random(int(self.env.trial_seed) * 7919 + int(time.time() * 1000) % 100000)
        if os.environ.get("DET_PRINT_UID"):  # agent user groups: which host account runs the trial
            print(f"trial process uid={os.getuid()} gid={os.getgid()}", flush=True)

    @staticmethod
    def from_trial(trial_inst: Any, context: Any, env: Any, workloads: Any, load_path: Any, rendezvous_info: Any,
                   dist_config: Any) -> "NoOpTrialController":
        return NoOpTrialController(context, env, workloads, load_path, rendezvous_info, dist_config)

    def _chaos(self, which: str) -> None:
        hp = self.context.get_hparams()
        p = float(hp.get(f"chaos_probability_{which}", hp.get("chaos_probability", 0.0)))
        if p > 0 and self.chaos.random() < p:
            raise RuntimeError(f"CHAOS! failing in {which}")

    def _step_metric(self) -> float:
        prog = self.context.get_hparams().get("metrics_progression", "decreasing")
        if prog == "decreasing":
            self.metric *= 0.9
        elif prog == "increasing":
            self.metric = 1.0 - (1.0 - self.metric) * 0.9
        return self.metric

    def train_for_step(self, step_id: int, num_batches: int) -> Dict[str, Any]:
        self._chaos("train")
        time.sleep(float(self.context.get_hparams().get("sleep", 0.0)))
        n = int(self.context.get_hparams().get("log_lines", 0))
        if n:
            t0, span = time.time(), float(self.context.get_hparams().get("log_seconds", 0.0))
            for i in range(n):
                print(f"spam step={step_id} line={i}", flush=True)
                if span and i % 100 == 99:
                    time.sleep(max(0.0, t0 + span * (i + 1) / n - time.time()))
        self.trained_steps += 1
        m = self._step_metric()
        print(f"finished train_batch for rank {self.context.distributed.get_rank()}", flush=True)
        return {"batch_metrics": [{"loss": m} for _ in range(num_batches)], "avg_metrics": {"loss": m},
                "num_inputs": num_batches * self.context.get_per_slot_batch_size()}

    def compute_validation_metrics(self, step_id: int) -> Dict[str, Any]:
        hp = self.context.get_hparams()
        marker = pathlib.Path("/tmp", f"det-noop-failed-{self.env.det_cluster_id}-{self.env.det_experiment_id}-"
                                      f"{self.env.det_trial_id}")
        if hp.get("fail_on_first_validation") and not marker.exists():
            marker.write_text("1")  # survives the process restart
            raise RuntimeError("failing on first validation")
        self._chaos("validate")
        return {"validation_metrics": {"validation_error": self.metric}, "num_inputs": int(hp.get("validation_set_size", 32))}

    def save(self, path: pathlib.Path) -> None:
        if self.context.get_hparams().get("fail_on_checkpoint_save"):
            raise RuntimeError("failing on checkpoint save")
        self._chaos("checkpoint")
        path.mkdir(parents=True, exist_ok=True)
        path.joinpath(self.CHECKPOINT_FILENAME).write_text(
            json.dumps({"metric": self.metric, "trained_steps": self.trained_steps}))

    def load(self, path: pathlib.Path) -> None:
        d = json.loads(pathlib.Path(path).joinpath(self.CHECKPOINT_FILENAME).read_text())
        self.metric = d["metric"]
        self.trained_steps = d["trained_steps"]


class NoOpTrial(trial.Trial):
    trial_controller_class = NoOpTrialController

    def __init__(self, context: trial.TrialContext) -> None:
        self.context = context
