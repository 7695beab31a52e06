"""CIFAR-10 CNN trial (reference examples/computer_vision/cifar10_pytorch/model_def.py:42-122):
RMSprop, cross-entropy, the reference's three-conv-block network with dropout.

Data: CIFAR-10 cannot be downloaded here, so a learnable synthetic stand-in in CIFAR's own storage
layout (uint8 HWC images, class templates + noise) is used.  The reference decodes and normalises
per sample on the host (``ToTensor`` + ``Normalize((0.5,)*3, (0.5,)*3)``); here each batch arrives
as one uint8 tensor (no per-sample host work) and the same normalisation, (x/255 - 0.5)/0.5, runs
on the GPU in the ``u8_normalize`` HIP kernel inside ``train_batch`` -- so with
``optimizations.hip_graph`` it is part of the replayed graph.  On MI355X the network runs on the
native CNN kernels (``ops/cnn.py``; fp32 at O0, bf16 via ``configure_apex_amp`` at O2) and the loss
and accuracy come from one fused cross-entropy launch.
"""
from typing import Any, Dict

import torch
import torch.nn as nn

from determined_1_amd import pytorch
from determined_1_amd.models import CIFAR10CNN
from determined_1_amd.models.synthetic import SyntheticImageClasses, passthrough_collate
from determined_1_amd.ops.cnn import cross_entropy
from determined_1_amd.ops.functional import u8_normalize

MEAN = STD = (127.5, 127.5, 127.5)  # ToTensor (/255) then Normalize(0.5, 0.5)


class CIFARTrial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        # channels_last end to end: the uint8 NHWC batch normalises straight into NHWC and MIOpen's
        # NHWC implicit-GEMM convs run without the NCHW<->NHWC transpose kernels around every conv
        net = CIFAR10CNN(hp.get("layer1_dropout", 0.25), hp.get("layer2_dropout", 0.25), hp.get("layer3_dropout", 0.5))
        self.model = context.wrap_model(net.to(memory_format=torch.channels_last))
        self.opt = context.wrap_optimizer(torch.optim.RMSprop(
            self.model.parameters(), lr=hp.get("learning_rate", 1e-4), weight_decay=hp.get("learning_rate_decay", 1e-6),
            alpha=0.9))
        amp = hp.get("amp")
        if amp and amp != "O0":
            self.model, self.opt = context.configure_apex_amp(self.model, self.opt, opt_level=amp)
        self.loss = nn.CrossEntropyLoss()

    def build_training_data_loader(self) -> pytorch.DataLoader:
        n = int(self.context.get_hparams().get("train_records", 50000))  # CIFAR-10 train split size
        return pytorch.DataLoader(SyntheticImageClasses(n, 32), batch_size=self.context.get_per_slot_batch_size(),
                                  collate_fn=passthrough_collate)

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        n = int(self.context.get_hparams().get("validation_records", 10000))  # CIFAR-10 test split size
        return pytorch.DataLoader(SyntheticImageClasses(n, 32, seed=1),
                                  batch_size=self.context.get_per_slot_batch_size(), collate_fn=passthrough_collate)

    def _images(self, x_u8: torch.Tensor) -> torch.Tensor:
        dtype = next(self.model.parameters()).dtype
        return u8_normalize(x_u8.contiguous(), MEAN, STD, out_dtype=dtype)  # [N,C,H,W] channels_last

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        x, y = batch
        out = self.model(self._images(x))
        loss, acc, err = cross_entropy(out, y, with_accuracy=True, with_error=True)  # one fused launch on the GPU
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss, "train_error": err, "train_accuracy": acc}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        x, y = batch
        loss, acc, err = cross_entropy(self.model(self._images(x)), y, with_accuracy=True, with_error=True)
        return {"validation_loss": loss, "validation_error": err, "validation_accuracy": acc}
