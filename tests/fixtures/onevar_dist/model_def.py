"""Cluster-submittable model definition: the analytic one-variable trial (see tests/fixtures/onevar.py)
with a validation loader, used by the multi-slot (gloo DP through the harness launcher) e2e test."""
from typing import Any, Dict, Tuple

import torch

from determined_1_amd import pytorch


class OnesDataset(torch.utils.data.Dataset):
    def __len__(self) -> int:
        return 64

    def __getitem__(self, index: int) -> Tuple[torch.Tensor, torch.Tensor]:
        return torch.tensor([1.0]), torch.tensor([1.0])


class OneVarTrial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        model = torch.nn.Linear(1, 1, bias=False)
        model.weight.data.fill_(0)
        self.model = context.wrap_model(model)
        self.opt = context.wrap_optimizer(torch.optim.SGD(self.model.parameters(), float(context.get_hparams()["lr"])))
        self.loss_fn = torch.nn.MSELoss()

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, Any]:
        data, label = batch
        loss = self.loss_fn(self.model(data), label)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss, "weight": self.model.weight.detach().reshape(())}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        data, label = batch
        return {"val_loss": self.loss_fn(self.model(data), label),
                "weight": self.model.weight.detach().reshape(())}

    def build_training_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(OnesDataset(), batch_size=self.context.get_per_slot_batch_size())

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(OnesDataset(), batch_size=self.context.get_per_slot_batch_size())
