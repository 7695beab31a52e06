"""XOR trials with variations (metric reducers, callbacks, full-dataset eval, LR schedulers,
legacy interface).  Mirrors the coverage of the reference's pytorch_xor_model.py fixtures."""
from typing import Any, Dict

import numpy as np
import torch

from determined_1_amd import pytorch


def xor_data(n: int = 4):
    x = torch.tensor([[0.0, 0.0], [0.0, 1.0], [1.0, 0.0], [1.0, 1.0]]).repeat(n // 4, 1)
    y = torch.tensor([[0.0], [1.0], [1.0], [0.0]]).repeat(n // 4, 1)
    return torch.utils.data.TensorDataset(x, y)


class XORTrial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        torch.manual_seed(context.get_trial_seed())
        self.model = context.wrap_model(torch.nn.Sequential(
            torch.nn.Linear(2, int(hp.get("hidden_size", 8))), torch.nn.Sigmoid(),
            torch.nn.Linear(int(hp.get("hidden_size", 8)), 1), torch.nn.Sigmoid()))
        opt_name = hp.get("optimizer", "sgd")
        lr = float(hp.get("lr", 0.5))
        if opt_name == "adam":
            opt = torch.optim.Adam(self.model.parameters(), lr=lr)
        elif opt_name == "rmsprop":
            opt = torch.optim.RMSprop(self.model.parameters(), lr=lr)
        else:
            opt = torch.optim.SGD(self.model.parameters(), lr=lr, momentum=float(hp.get("momentum", 0.9)))
        self.opt = context.wrap_optimizer(opt)
        if hp.get("lr_schedule"):
            mode = pytorch.LRScheduler.StepMode[hp["lr_schedule"]]
            self.sched = context.wrap_lr_scheduler(torch.optim.lr_scheduler.StepLR(self.opt, 1, gamma=0.9), mode)
        self.dropout = torch.nn.Dropout(float(hp.get("dropout", 0.0)))

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, Any]:
        x, y = batch
        out = self.model(self.dropout(x))
        loss = torch.nn.functional.binary_cross_entropy(out, y)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss, "lr": self.opt.param_groups[0]["lr"]}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        x, y = batch
        out = self.model(x)
        loss = torch.nn.functional.binary_cross_entropy(out, y)
        acc = ((out > 0.5).float() == y).float().mean()
        return {"validation_loss": loss, "accuracy": acc, "binary_error": 1.0 - acc}

    def build_training_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(xor_data(64), batch_size=self.context.get_per_slot_batch_size(), shuffle=False)

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(xor_data(16), batch_size=self.context.get_per_slot_batch_size())


class XORTrialPerMetricReducers(XORTrial):
    def evaluation_reducer(self) -> Dict[str, pytorch.Reducer]:
        return {"validation_loss": pytorch.Reducer.AVG, "accuracy": pytorch.Reducer.MAX,
                "binary_error": pytorch.Reducer.MIN}


class XORTrialFullDataset(XORTrial):
    evaluate_batch = pytorch.PyTorchTrial.evaluate_batch  # type: ignore

    def evaluate_full_dataset(self, data_loader: torch.utils.data.DataLoader) -> Dict[str, Any]:
        losses = []
        for x, y in data_loader:
            x, y = self.context.to_device(x), self.context.to_device(y)
            losses.append(torch.nn.functional.binary_cross_entropy(self.model(x), y).item())
        return {"validation_loss": float(np.mean(losses))}


class Counter(pytorch.PyTorchCallback):
    def __init__(self) -> None:
        self.validation_starts = 0
        self.validation_ends = 0
        self.checkpoints = 0

    def on_validation_start(self) -> None:
        self.validation_starts += 1

    def on_validation_end(self, metrics: Dict[str, Any]) -> None:
        self.validation_ends += 1
        self.last_metrics = metrics

    def on_checkpoint_end(self, checkpoint_dir: str) -> None:
        self.checkpoints += 1

    def state_dict(self) -> Dict[str, Any]:
        return {"validation_starts": self.validation_starts, "validation_ends": self.validation_ends,
                "checkpoints": self.checkpoints}

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        self.validation_starts = state_dict["validation_starts"]
        self.validation_ends = state_dict["validation_ends"]
        self.checkpoints = state_dict["checkpoints"]


class XORTrialCallbacks(XORTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        super().__init__(context)
        self.counter = Counter()

    def build_callbacks(self) -> Dict[str, pytorch.PyTorchCallback]:
        return {"counter": self.counter}


class XORTrialLegacy(pytorch.PyTorchTrial):
    """Deprecated build_model()/optimizer() interface."""

    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context

    def build_model(self) -> torch.nn.Module:
        torch.manual_seed(0)
        return torch.nn.Sequential(torch.nn.Linear(2, 8), torch.nn.Sigmoid(), torch.nn.Linear(8, 1),
                                   torch.nn.Sigmoid())

    def optimizer(self, model: torch.nn.Module) -> torch.optim.Optimizer:
        return torch.optim.SGD(model.parameters(), lr=0.5)

    def train_batch(self, batch: Any, model: torch.nn.Module, epoch_idx: int, batch_idx: int) -> Any:  # type: ignore
        x, y = batch
        return {"loss": torch.nn.functional.binary_cross_entropy(model(x), y)}

    def evaluate_batch(self, batch: Any, model: torch.nn.Module) -> Dict[str, Any]:  # type: ignore
        x, y = batch
        return {"validation_loss": torch.nn.functional.binary_cross_entropy(model(x), y)}

    def build_training_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(xor_data(64), batch_size=self.context.get_per_slot_batch_size())

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(xor_data(16), batch_size=self.context.get_per_slot_batch_size())
