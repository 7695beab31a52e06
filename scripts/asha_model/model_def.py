"""The CIFAR-10 ASHA trial with its GPU time MODELLED (scripts/bench_asha.py --modelled-batch-ms).

The 16-trial adaptive_asha benchmark (BASELINE north-star #2, reference
examples/computer_vision/cifar10_pytorch/adaptive.yaml) is 32 epochs x 50,000 records per full trial.
On CPU artificial slots the real CNN would take hours; its MI355X cost is known (0.289 ms per batch of
32 with the native kernels, README), so each train_batch here waits that long instead -- scaled by the
trial's sampled batch size -- and the master, agent, scheduler, searcher, container starts and the
harness's workload loop are all the real ones.  What the benchmark then measures is the control
plane: how much slot time is lost to anything but (modelled) training.

The waits are paced against a running clock and slept in >= 2 ms pieces (time.sleep of 0.3 ms
would overshoot by its own latency); host work the harness does per batch counts toward the modelled
time, as it would overlap a GPU step on the real box.
"""
import os
import time
from typing import Any, Dict

import torch

from determined_1_amd import pytorch

BATCH_MS = float(os.environ.get("DET_MODEL_BATCH_MS", "0.289"))  # at batch 32
EVAL_FRACTION = 0.35  # forward-only validation batch / training batch


class _Pace:
    def __init__(self) -> None:
        self.t = time.perf_counter()

    def advance(self, seconds: float) -> None:
        self.t += seconds
        lag = self.t - time.perf_counter()
        if lag > 0.002:
            time.sleep(lag)
        elif lag < -0.02:  # host work ran past the model: do not bank the difference
            self.t = time.perf_counter()


def _scaled(bs: int) -> float:
    return BATCH_MS * (0.5 + 0.5 * bs / 32.0) / 1e3


class ModelledCIFARTrial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        self.model = context.wrap_model(torch.nn.Linear(4, 10))
        self.opt = context.wrap_optimizer(torch.optim.SGD(self.model.parameters(),
                                                          lr=float(context.get_hparam("learning_rate"))))
        bs = context.get_per_slot_batch_size()
        self.train_s = _scaled(bs)
        self.eval_s = EVAL_FRACTION * _scaled(bs)
        self.pace = _Pace()
        self.lr = float(context.get_hparam("learning_rate"))

    def _data(self, n: int) -> pytorch.DataLoader:
        ds = torch.utils.data.TensorDataset(torch.zeros(n, 4), torch.zeros(n, dtype=torch.int64))
        return pytorch.DataLoader(ds, batch_size=self.context.get_per_slot_batch_size())

    def build_training_data_loader(self) -> pytorch.DataLoader:
        return self._data(50000)

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        return self._data(int(self.context.get_hparams().get("validation_records", 10000)))

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, Any]:
        self.pace.advance(self.train_s)
        return {"loss": 1.0}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        self.pace.advance(self.eval_s)
        # a validation error that depends on the sampled hparams: ASHA's promotions are hparam-driven
        return {"validation_error": abs(self.lr - 1e-2) / (1.0 + abs(self.lr))}
