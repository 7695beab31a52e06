"""GAEA searched-cell ImageNet evaluation (reference examples/nas/gaea_pytorch/eval):
the networks and helpers come from the ``determined_1_amd.models.gaea`` library

This file is the experiment's user code (it is what a checkpoint's ``code/`` holds): the
Trial -- data, optimizer, training and evaluation steps -- lives here; the network building
blocks are imported from the framework's model library, as the reference examples import theirs
from torchvision / transformers.
"""
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch

from determined_1_amd.models.synthetic import SyntheticClassification
from determined_1_amd import pytorch as det_torch
from determined_1_amd.models.darts import OPS, PRIMITIVES, FactorizedReduce, ReLUConvBN, drop_path, topk_accuracy
from determined_1_amd.models.gaea import ACTIVATIONS, EMAModel, GAEA_IMAGENET_GENOTYPE, NetworkImageNet, label_smoothing_ce, lr_multiplier


class GAEAEvalTrial(det_torch.PyTorchTrial):
    def __init__(self, context: det_torch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        self.hp = hp
        self.num_classes = int(hp.get("num_classes", 1000))
        self.image_size = int(hp.get("image_size", 224))
        genotype = hp.get("genotype") or GAEA_IMAGENET_GENOTYPE
        net = NetworkImageNet(genotype, ACTIVATIONS[str(hp.get("activation", "swish"))], int(hp.get("init_channels", 48)),
                              self.num_classes, int(hp.get("layers", 14)), bool(hp.get("auxiliary", False)),
                              bool(hp.get("do_SE", True)), float(hp.get("drop_path_prob", 0.2)),
                              float(hp.get("drop_prob", 0.2)))
        self.ema = EMAModel(net, float(hp.get("ema_decay", 0.999)))
        self.model = context.wrap_model(self.ema)
        self.opt = context.wrap_optimizer(torch.optim.SGD(net.parameters(), lr=float(hp.get("learning_rate", 0.5)),
                                                          momentum=float(hp.get("momentum", 0.9)),
                                                          weight_decay=float(hp.get("weight_decay", 3e-5))))
        kind = str(hp.get("lr_scheduler", "linear"))
        warm, max_ep = int(hp.get("warmup_epochs", 5)), int(hp.get("lr_epochs", 300))
        gamma, every = float(hp.get("lr_gamma", 0.97)), int(hp.get("lr_decay_every", 2))
        self.sched = torch.optim.lr_scheduler.LambdaLR(
            self.opt, lambda e: lr_multiplier(kind, e, warm, max_ep, gamma, every))
        context.wrap_lr_scheduler(self.sched, det_torch.LRScheduler.StepMode.STEP_EVERY_EPOCH)
        self.smooth = float(hp.get("label_smoothing_rate", 0.1))
        self.clip = float(hp.get("clip_gradients_l2_norm", 5.0))

    def _data(self, n: int, seed: int) -> SyntheticClassification:
        return SyntheticClassification(n, (3, self.image_size, self.image_size), num_classes=self.num_classes, seed=seed)

    def build_training_data_loader(self) -> det_torch.DataLoader:
        return det_torch.DataLoader(self._data(int(self.hp.get("train_records", 1281167)), 0),
                                    batch_size=self.context.get_per_slot_batch_size(), shuffle=True, drop_last=True)

    def build_validation_data_loader(self) -> det_torch.DataLoader:
        return det_torch.DataLoader(self._data(int(self.hp.get("validation_records", 50000)), 1),
                                    batch_size=self.context.get_per_slot_batch_size())

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, Any]:
        self.ema.update()
        x, y = batch
        logits, logits_aux = self.model(x)
        loss = label_smoothing_ce(logits, y, self.smooth)
        if logits_aux is not None:
            loss = loss + float(self.hp.get("auxiliary_weight", 0.4)) * label_smoothing_ce(logits_aux, y, self.smooth)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt, clip_grads=det_torch.ClipGradsNorm(self.clip) if self.clip > 0 else None)
        top1, top5 = topk_accuracy(logits, y)
        return {"loss": loss, "top1_accuracy": top1, "top5_accuracy": top5}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        x, y = batch
        logits, _ = self.model(x)
        top1, top5 = topk_accuracy(logits, y)
        out = {"loss": label_smoothing_ce(logits, y, self.smooth), "top1_accuracy": top1, "top5_accuracy": top5}
        self.ema.swap()
        try:
            logits, _ = self.model(x)
        finally:
            self.ema.swap()
        top1, top5 = topk_accuracy(logits, y)
        out.update({"ema_loss": label_smoothing_ce(logits, y, self.smooth), "top1_ema": top1, "top5_ema": top5})
        return out

