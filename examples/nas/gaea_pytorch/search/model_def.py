"""GAEA weight-sharing architecture search (reference examples/nas/gaea_pytorch/search):
the networks and helpers come from the ``determined_1_amd.models.gaea`` library

This file is the experiment's user code (it is what a checkpoint's ``code/`` holds): the
Trial -- data, optimizer, training and evaluation steps -- lives here; the network building
blocks are imported from the framework's model library, as the reference examples import theirs
from torchvision / transformers.
"""
import logging
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from determined_1_amd.models.synthetic import SyntheticClassification
from determined_1_amd import pytorch as det_torch
from determined_1_amd.models.darts import OPS, PRIMITIVES, FactorizedReduce, ReLUConvBN, drop_path, topk_accuracy
from determined_1_amd.models.gaea import BilevelPairs, EG, SearchNetwork


class _GenotypeLogger(det_torch.PyTorchCallback):
    def __init__(self, net: SearchNetwork) -> None:
        self.net = net
        self.last = None  # type: Optional[Dict[str, Any]]

    def on_validation_end(self, metrics: Dict[str, Any]) -> None:
        self.last = self.net.genotype()
        logging.info(f"genotype: {self.last}")



class GAEASearchTrial(det_torch.PyTorchTrial):
    def __init__(self, context: det_torch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        self.hp = hp
        self.net = SearchNetwork(int(hp.get("init_channels", 16)), int(hp.get("n_classes", 10)),
                                 int(hp.get("layers", 8)), int(hp.get("nodes", 4)), k=int(hp.get("shuffle_factor", 4)))
        self.model = context.wrap_model(self.net)
        self.ws_opt = context.wrap_optimizer(torch.optim.SGD(self.net.ws_parameters(), float(hp.get("learning_rate", 0.1)),
                                                             momentum=float(hp.get("momentum", 0.9)),
                                                             weight_decay=float(hp.get("weight_decay", 3e-4))))
        self.arch_opt = context.wrap_optimizer(EG(self.net.arch_parameters(), float(hp.get("arch_learning_rate", 0.1))))
        context.wrap_lr_scheduler(torch.optim.lr_scheduler.CosineAnnealingLR(
            self.ws_opt, int(hp.get("scheduler_epochs", 50)), float(hp.get("min_learning_rate", 0.0))),
            det_torch.LRScheduler.StepMode.STEP_EVERY_EPOCH)
        self.genotype_cb = _GenotypeLogger(self.net)
        self.train_data = None  # type: Optional[BilevelPairs]
        self.last_epoch = 0

    def build_callbacks(self) -> Dict[str, det_torch.PyTorchCallback]:
        return {"genotype": self.genotype_cb}

    def build_training_data_loader(self) -> det_torch.DataLoader:
        n = int(self.hp.get("train_records", 50000))
        self.train_data = BilevelPairs(SyntheticClassification(n, (3, 32, 32)))
        return det_torch.DataLoader(self.train_data, batch_size=self.context.get_per_slot_batch_size(), shuffle=True,
                                    drop_last=True)

    def build_validation_data_loader(self) -> det_torch.DataLoader:
        n = int(self.hp.get("validation_records", 10000))
        return det_torch.DataLoader(SyntheticClassification(n, (3, 32, 32), seed=1),
                                    batch_size=self.context.get_per_slot_batch_size())

    def _trainable(self, arch: bool) -> None:
        for p in self.net.arch_parameters():
            p.requires_grad_(arch)
        for p in self.net.ws_parameters():
            p.requires_grad_(not arch)

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, Any]:
        if epoch_idx != self.last_epoch and self.train_data is not None:
            self.train_data.shuffle_val()
        self.last_epoch = epoch_idx
        x_train, y_train, x_val, y_val = batch
        self._trainable(arch=False)
        loss = F.cross_entropy(self.model(x_train), y_train)
        self.context.backward(loss)
        self.context.step_optimizer(self.ws_opt)
        self._trainable(arch=True)
        arch_loss = F.cross_entropy(self.model(x_val), y_val)
        self.context.backward(arch_loss)
        self.context.step_optimizer(self.arch_opt)
        self._trainable(arch=False)
        return {"loss": loss, "arch_loss": arch_loss}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        x, y = batch
        logits = self.model(x)
        top1, top5 = topk_accuracy(logits, y)
        return {"loss": F.cross_entropy(logits, y), "top1_accuracy": top1, "top5_accuracy": top5}


# ------------------------------------------------------------------------------------------------
# evaluation network (ImageNet)
# ------------------------------------------------------------------------------------------------

