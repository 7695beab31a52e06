"""RetinaNet R50-FPN detection (reference ``examples/computer_vision/mmdetection_pytorch`` with
``retinanet.yaml``, which wraps mmdetection's ``retinanet_r50_fpn_1x_coco``): 2 images per GPU, SGD
lr 0.01 per 16 images with momentum 0.9 and weight decay 1e-4, linear warmup over the first 500
iterations, focal + L1 losses.  Validation reports the mean best box IoU over ground-truth boxes.

mmdetection is not in this image; the model is the framework's own ``models.retinanet`` (device
NMS, padded batch shapes bucketed so MIOpen's find-db covers every conv shape).  Data: synthetic
COCO-shaped instances (``models.detection.SyntheticCocoInstances``); weights random-init.
"""
from typing import Any, Dict

import torch

from determined_1_amd import pytorch
from determined_1_amd.models.detection import SyntheticCocoInstances, list_collate
from determined_1_amd.models.faster_rcnn import box_iou
from determined_1_amd.models.retinanet import RetinaNet


class RetinaNetTrial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        self.hp = hp
        self.num_classes = int(hp.get("num_classes", 81))
        model = RetinaNet(num_classes=self.num_classes, min_size=int(hp.get("transform_min_size", 800)),
                          max_size=int(hp.get("transform_max_size", 1333)), arch=hp.get("backbone", "resnet50"),
                          size_divisible=int(hp.get("size_divisible", 128)))
        self.model = context.wrap_model(model)
        lr = float(hp.get("lr_per_16_images", 0.01)) * context.get_global_batch_size() / 16.0
        self.optimizer = context.wrap_optimizer(torch.optim.SGD(
            [p for p in self.model.parameters() if p.requires_grad], lr=lr, momentum=float(hp.get("momentum", 0.9)),
            weight_decay=float(hp.get("weight_decay", 1e-4))))
        warm = int(hp.get("warmup_iters", 500))
        ratio = float(hp.get("warmup_ratio", 0.001))
        self.lr_scheduler = context.wrap_lr_scheduler(
            torch.optim.lr_scheduler.LambdaLR(self.optimizer, lambda it: 1.0 if it >= warm
                                              else ratio + (1.0 - ratio) * it / warm),
            step_mode=pytorch.LRScheduler.StepMode.STEP_EVERY_BATCH)
        amp = hp.get("amp")
        if amp and amp != "O0":
            self.model, self.optimizer = context.configure_apex_amp(self.model, self.optimizer, opt_level=amp)

    def _data(self, train: bool) -> SyntheticCocoInstances:
        n = int(self.hp.get("train_records" if train else "validation_records", 1000 if train else 16))
        return SyntheticCocoInstances(n, num_classes=self.num_classes, min_size=int(self.hp.get("min_image_size", 480)),
                                      max_size=int(self.hp.get("max_image_size", 640)), seed=0 if train else 1,
                                      instance_dist=str(self.hp.get("instance_dist", "uniform")))

    def build_training_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(self._data(True), batch_size=self.context.get_per_slot_batch_size(),
                                  collate_fn=list_collate, shuffle=True, num_workers=int(self.hp.get("num_workers", 0)))

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(self._data(False), batch_size=self.context.get_per_slot_batch_size(),
                                  collate_fn=list_collate, num_workers=int(self.hp.get("num_workers", 0)))

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        images, targets = batch
        losses = self.model(list(images), list(targets))
        loss = sum(losses.values())
        self.context.backward(loss)
        self.context.step_optimizer(self.optimizer)
        return {"loss": loss.detach(), **{k: v.detach() for k, v in losses.items()}}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        images, targets = batch
        out = self.model(list(images))
        s, n = 0.0, 0
        for o, t in zip(out, targets):
            gb = t["boxes"].float()
            n += gb.shape[0]
            if o["boxes"].numel():
                s += float(box_iou(gb, o["boxes"].float().to(gb.device)).max(1).values.sum())
        return {"val_box_iou": s / max(n, 1)}
