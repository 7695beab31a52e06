"""ResNet-50 ImageNet-shape PyTorchTrial: the north-star benchmark trial (BASELINE.md:
"ResNet-50 samples/s (whole node) at 1/2/4/8 MI355X ... bf16, SGD-momentum"); bench.py runs this
class.

Per batch: uint8 NHWC images (pinned, DMA'd ahead by the DevicePrefetcher) -> ``u8_normalize``
HIP kernel -> bf16 channels_last tensor -> ResNet-50 forward/backward entirely on the hand-written
HIP kernels (stem patch conv, 1x1 GEMMs and 3x3 implicit GEMMs with the BatchNorm statistics /
apply / backward partials fused into their prologues and epilogues, max/avg pool, head; no MIOpen
call in the step: profiles/r5_resnet50_steady_final.txt) -> fused arena SGD-momentum HIP kernel,
with gradient buckets reduced over RCCL during backward when ``slots_per_trial > 1``.

Hyperparameters: ``global_batch_size``, ``lr``, ``momentum``, ``weight_decay``, ``arch``,
``amp`` (O0/O1/O2), ``channels_last``, ``num_classes``, ``image_size``, ``fused_bn``,
``native_conv1x1``.

This file is the experiment's user code (it is what a checkpoint's ``code/`` holds); the network
comes from the framework's model library, as the reference examples import theirs from
torchvision.
"""
from typing import Any, Dict

import torch
import torch.nn as nn

from determined_1_amd import pytorch as det_torch
from determined_1_amd.models import resnet
from determined_1_amd.models.synthetic import IMAGENET_MEAN, IMAGENET_STD, SyntheticImages, passthrough_collate
from determined_1_amd.ops.functional import u8_normalize


class ResNetImageNetTrial(det_torch.PyTorchTrial):
    def __init__(self, context: det_torch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        arch = hp.get("arch", "resnet50")
        self.num_classes = int(hp.get("num_classes", 1000))
        self.image_size = int(hp.get("image_size", 224))
        self.channels_last = bool(hp.get("channels_last", True))
        resnet.FUSED_BN = bool(hp.get("fused_bn", True))
        resnet.NATIVE_CONV1X1 = bool(hp.get("native_conv1x1", True))
        resnet.BN_PROLOGUE = bool(hp.get("bn_prologue", False))
        resnet.NATIVE_STEM = bool(hp.get("native_stem", True))
        resnet.NATIVE_CONV3X3 = bool(hp.get("native_conv3x3", True))
        model = getattr(resnet, arch)(num_classes=self.num_classes)
        if self.channels_last:
            model = model.to(memory_format=torch.channels_last)
        self.model = context.wrap_model(model)
        if self.channels_last:
            self.model.to(memory_format=torch.channels_last)
        self.opt = context.wrap_optimizer(torch.optim.SGD(
            self.model.parameters(), lr=float(hp.get("lr", 0.1)), momentum=float(hp.get("momentum", 0.9)),
            weight_decay=float(hp.get("weight_decay", 5e-5)), nesterov=bool(hp.get("nesterov", False))))
        amp = hp.get("amp", "O1")
        if amp and amp != "O0":
            self.model, self.opt = context.configure_apex_amp(self.model, self.opt, opt_level=amp)
        self.loss_fn = nn.CrossEntropyLoss()
        self.compute_dtype = torch.bfloat16 if amp and amp != "O0" else torch.float32

    def _inputs(self, images_u8: torch.Tensor) -> torch.Tensor:
        if images_u8.dtype == torch.uint8:
            # the native stem reads 4-channel pixels (8 B): the normalize kernel pads for free
            pad4 = self.channels_last and resnet.NATIVE_STEM and resnet.FUSED_BN and images_u8.is_cuda
            x = u8_normalize(images_u8, IMAGENET_MEAN, IMAGENET_STD, out_dtype=self.compute_dtype, pad4=pad4)
            return x if self.channels_last else x.contiguous()
        return images_u8

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        images, labels = batch
        out = self.model(self._inputs(images))
        loss = self.loss_fn(out.float(), labels)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        images, labels = batch
        out = self.model(self._inputs(images)).float()
        loss = self.loss_fn(out, labels)
        acc = (out.argmax(1) == labels).float().mean()
        return {"validation_loss": loss, "accuracy": acc}

    def build_training_data_loader(self) -> det_torch.DataLoader:
        bs = self.context.get_per_slot_batch_size()
        n = int(self.context.get_hparams().get("train_records", 1281167))
        ds = SyntheticImages(n, self.image_size, num_classes=self.num_classes, pool=max(2 * bs, 64))
        return det_torch.DataLoader(ds, batch_size=bs, collate_fn=passthrough_collate, drop_last=True)

    def build_validation_data_loader(self) -> det_torch.DataLoader:
        bs = self.context.get_per_slot_batch_size()
        n = int(self.context.get_hparams().get("validation_records", 4 * bs))
        ds = SyntheticImages(n, self.image_size, num_classes=self.num_classes, pool=max(bs, 64), seed=1)
        return det_torch.DataLoader(ds, batch_size=bs, collate_fn=passthrough_collate)

