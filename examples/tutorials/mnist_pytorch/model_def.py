"""MNIST CNN tutorial trial (reference examples/tutorials/mnist_pytorch/model_def.py): Adadelta,
NLL loss, per-batch accuracy; synthetic 28x28 class-template data instead of the MNIST download."""
from typing import Any, Dict

import torch
import torch.nn.functional as F

from determined_1_amd import pytorch
from determined_1_amd.models import MNISTNet
from determined_1_amd.models.synthetic import SyntheticClassification


class MNistTrial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        self.model = context.wrap_model(MNISTNet(hp.get("n_filters1", 32), hp.get("n_filters2", 64),
                                                 hp.get("dropout1", 0.25), hp.get("dropout2", 0.5)))
        self.opt = context.wrap_optimizer(torch.optim.Adadelta(self.model.parameters(), lr=hp.get("learning_rate", 1.0)))

    def build_training_data_loader(self) -> pytorch.DataLoader:
        ds = SyntheticClassification(int(self.context.get_hparams().get("train_records", 60000)), (1, 28, 28), noise=2.0)
        return pytorch.DataLoader(ds, batch_size=self.context.get_per_slot_batch_size(), shuffle=True)

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        ds = SyntheticClassification(int(self.context.get_hparams().get("validation_records", 10000)), (1, 28, 28),
                                    noise=2.0, seed=1)
        return pytorch.DataLoader(ds, batch_size=self.context.get_per_slot_batch_size())

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        data, labels = batch
        out = self.model(data)
        loss = F.nll_loss(out, labels)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss, "train_error": 1.0 - (out.argmax(1) == labels).float().mean()}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        data, labels = batch
        out = self.model(data)
        return {"validation_loss": F.nll_loss(out, labels),
                "accuracy": (out.argmax(1) == labels).float().mean()}
