"""DARTS CIFAR-10 architecture search as hyperparameter search (reference
examples/hp_search_benchmarks/darts_cifar10_pytorch): the networks and helpers come from the ``determined_1_amd.models.darts`` library

This file is the experiment's user code (it is what a checkpoint's ``code/`` holds): the
Trial -- data, optimizer, training and evaluation steps -- lives here; the network building
blocks are imported from the framework's model library, as the reference examples import theirs
from torchvision / transformers.
"""
from typing import Any, Callable, Dict, List, Sequence, Tuple

import torch
import torch.nn.functional as F

from determined_1_amd.models.synthetic import SyntheticClassification
from determined_1_amd import pytorch as det_torch
from determined_1_amd.models.darts import DARTSNetwork, genotype_from_hparams, topk_accuracy


class DARTSCNNTrial(det_torch.PyTorchTrial):
    def __init__(self, context: det_torch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        g = genotype_from_hparams(hp)
        self.epochs = int(hp.get("train_epochs", 300))
        self.net = DARTSNetwork(int(hp.get("init_channels", 36)), 10, int(hp.get("layers", 20)),
                                bool(hp.get("auxiliary", True)), g["normal"], g["reduce"])
        self.model = context.wrap_model(self.net)
        self.opt = context.wrap_optimizer(torch.optim.SGD(self.model.parameters(), lr=float(hp.get("learning_rate", 0.025)),
                                                          momentum=float(hp.get("momentum", 0.9)),
                                                          weight_decay=float(hp.get("weight_decay", 3e-4))))
        self.sched = torch.optim.lr_scheduler.CosineAnnealingLR(self.opt, self.epochs)
        context.wrap_lr_scheduler(self.sched, det_torch.LRScheduler.StepMode.STEP_EVERY_EPOCH)
        self.clip = float(hp.get("clip_gradients_l2_norm", 5.0))

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        x, y = batch
        hp = self.context.get_hparams()
        self.net.drop_path_prob = float(hp.get("drop_path_prob", 0.2)) * self.sched.last_epoch / max(1, self.epochs)
        logits, logits_aux = self.model(x)
        loss = F.cross_entropy(logits, y)
        if logits_aux is not None:
            loss = loss + float(hp.get("auxiliary_weight", 0.4)) * F.cross_entropy(logits_aux, y)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt, clip_grads=det_torch.ClipGradsNorm(self.clip) if self.clip > 0 else None)
        top1, top5 = topk_accuracy(logits, y)
        return {"loss": loss, "top1_accuracy": top1, "top5_accuracy": top5}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        x, y = batch
        logits, _ = self.model(x)
        top1, top5 = topk_accuracy(logits, y)
        return {"loss": F.cross_entropy(logits, y), "top1_accuracy": top1, "top5_accuracy": top5}

    def build_training_data_loader(self) -> det_torch.DataLoader:
        n = int(self.context.get_hparams().get("train_records", 50000))
        return det_torch.DataLoader(SyntheticClassification(n, (3, 32, 32)), batch_size=self.context.get_per_slot_batch_size(),
                                    shuffle=True, drop_last=True)

    def build_validation_data_loader(self) -> det_torch.DataLoader:
        n = int(self.context.get_hparams().get("validation_records", 10000))
        return det_torch.DataLoader(SyntheticClassification(n, (3, 32, 32), seed=1),
                                    batch_size=self.context.get_per_slot_batch_size())

