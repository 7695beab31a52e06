"""Object-detection fine-tuning with Faster R-CNN ResNet-50-FPN (reference
``examples/computer_vision/fasterrcnn_coco_pytorch/model_def.py``): a 2-class detector (background
+ pedestrian), SGD with momentum and weight decay, StepLR(3, 0.1) per epoch, an 80/20 train /
validation split, the reference's training signal (it back-propagates ``loss_box_reg``) and its
validation metric ``val_avg_iou`` -- the mean over ground-truth boxes of the best IoU among the
predictions that survive NMS at 0.1.

Data: the PennFudan download is unavailable offline, so a deterministic synthetic pedestrian-shaped
set stands in (PennFudan-sized images of 300-500 px with 1-4 upright boxes; ``data.py``).  Weights
are random-init (the reference fine-tunes COCO-pretrained weights, which cannot be fetched here).

MI355X path: RoIAlign over all FPN levels is one NHWC HIP kernel launch and every NMS runs on the
device (``determined_1_amd.ops.detect``); the backbone's frozen BatchNorm is folded into its convs.
"""
import copy
from typing import Any, Dict

import torch

from determined_1_amd import pytorch
from determined_1_amd.models.faster_rcnn import FasterRCNN, box_iou
from determined_1_amd.ops.detect import nms

from data import SyntheticPedestrians, collate_fn


class ObjectDetectionTrial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        n = int(hp.get("num_images", 170))  # PennFudan has 170 images
        dataset = SyntheticPedestrians(n, min_size=int(hp.get("min_image_size", 300)),
                                       max_size=int(hp.get("max_image_size", 500)))
        train_size = int(0.8 * len(dataset))
        self.dataset_train, self.dataset_val = torch.utils.data.random_split(
            dataset, [train_size, len(dataset) - train_size], generator=torch.Generator().manual_seed(0))
        model = FasterRCNN(num_classes=2, min_size=int(hp.get("transform_min_size", 800)),
                           max_size=int(hp.get("transform_max_size", 1333)), arch=hp.get("backbone", "resnet50"),
                           size_divisible=int(hp.get("size_divisible", 128)))
        self.model = context.wrap_model(model)
        self.optimizer = context.wrap_optimizer(torch.optim.SGD(
            [p for p in self.model.parameters() if p.requires_grad], lr=float(hp["learning_rate"]),
            momentum=float(hp["momentum"]), weight_decay=float(hp["weight_decay"])))
        self.lr_scheduler = context.wrap_lr_scheduler(
            torch.optim.lr_scheduler.StepLR(self.optimizer, step_size=3, gamma=0.1),
            step_mode=pytorch.LRScheduler.StepMode.STEP_EVERY_EPOCH)
        amp = hp.get("amp")
        if amp and amp != "O0":
            self.model, self.optimizer = context.configure_apex_amp(self.model, self.optimizer, opt_level=amp)

    def build_training_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(self.dataset_train, batch_size=self.context.get_per_slot_batch_size(),
                                  collate_fn=collate_fn)

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(self.dataset_val, batch_size=self.context.get_per_slot_batch_size(),
                                  collate_fn=collate_fn)

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        images, targets = batch
        loss_dict = self.model(list(images), list(targets))
        self.context.backward(loss_dict["loss_box_reg"])
        self.context.step_optimizer(self.optimizer)
        return {"loss": loss_dict["loss_box_reg"].detach(),
                **{k: v.detach() for k, v in loss_dict.items()}}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        images, targets = batch
        output = self.model(list(images), copy.deepcopy(list(targets)))
        sum_iou, num_boxes = 0.0, 0
        for idx, target in enumerate(targets):
            boxes, scores = output[idx]["boxes"], output[idx]["scores"]
            boxes = boxes[nms(boxes, scores, 0.1)]
            if boxes.numel():
                sum_iou += float(box_iou(target["boxes"].float(), boxes).max(1).values.sum())
            num_boxes += len(target["boxes"])
        return {"val_avg_iou": sum_iou / max(num_boxes, 1)}
