"""CIFAR-10 CNN trial (reference examples/computer_vision/cifar10_pytorch/model_def.py:42-122):
RMSprop, cross-entropy, epoch-based LR decay; synthetic 32x32x3 class-template data.  On MI355X
the trial runs bf16 via ``configure_apex_amp`` when ``amp`` is set."""
from typing import Any, Dict

import torch
import torch.nn as nn

from determined_1_amd import pytorch
from determined_1_amd.models import CIFAR10CNN
from determined_1_amd.models.synthetic import SyntheticClassification


class CIFARTrial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        self.model = context.wrap_model(CIFAR10CNN(hp.get("layer1_dropout", 0.25), hp.get("layer2_dropout", 0.25),
                                                   hp.get("layer3_dropout", 0.5)))
        self.opt = context.wrap_optimizer(torch.optim.RMSprop(
            self.model.parameters(), lr=hp.get("learning_rate", 1e-4), weight_decay=hp.get("learning_rate_decay", 1e-6)))
        amp = hp.get("amp")
        if amp and amp != "O0":
            self.model, self.opt = context.configure_apex_amp(self.model, self.opt, opt_level=amp)
        self.loss = nn.CrossEntropyLoss()

    def build_training_data_loader(self) -> pytorch.DataLoader:
        # in-memory synthetic data: batched __getitems__ is cheaper than worker-process IPC
        ds = SyntheticClassification(50000, (3, 32, 32), noise=3.0)
        return pytorch.DataLoader(ds, batch_size=self.context.get_per_slot_batch_size(), shuffle=True)

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        ds = SyntheticClassification(10000, (3, 32, 32), noise=3.0, seed=1)
        return pytorch.DataLoader(ds, batch_size=self.context.get_per_slot_batch_size())

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        x, y = batch
        out = self.model(x)
        loss = self.loss(out.float(), y)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss, "train_error": 1.0 - (out.argmax(1) == y).float().mean()}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        x, y = batch
        out = self.model(x).float()
        err = 1.0 - (out.argmax(1) == y).float().mean()
        return {"validation_loss": self.loss(out, y), "validation_error": err, "validation_accuracy": 1.0 - err}
