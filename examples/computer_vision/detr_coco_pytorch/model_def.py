"""DETR on COCO-shaped data (reference ``examples/computer_vision/detr_coco_pytorch/model_def.py``):
AdamW with a separate backbone learning rate, StepLR stepped every epoch, gradient-norm clipping,
the weighted sum of DETR's set losses (final + aux decoder layers) as the training loss, and a
full-dataset evaluation returning the averaged losses plus COCO bbox mAP stats.

Data: COCO cannot be downloaded here, so ``backend: fake`` (the reference's own no-download mode)
serves deterministic synthetic COCO-shaped samples -- variable-size images with 1-6 coloured
objects, padded per batch with a mask (``determined_1_amd.models.detection.SyntheticDetection``).
The evaluator is the numpy COCO-protocol implementation in the same module (pycocotools is not
installed).

MI355X notes: the backbone's frozen BatchNorm is folded into its convolutions (one conv per
layer), the matcher moves all decoder layers' cost matrices to the host in one copy per step, and
``clip_grads`` uses the fused gradient-norm kernel (``det.pytorch.ClipGradsNorm``).
"""
import functools
from collections import defaultdict
from typing import Any, Dict

import torch

from determined_1_amd import pytorch
from determined_1_amd.models import detr
from determined_1_amd.models.detection import CocoBboxEvaluator, SyntheticDetection, box_cxcywh_to_xyxy, pad_collate, postprocess


class DETRTrial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        self.hp = context.get_hparams()
        if self.hp.get("backend", "fake") != "fake":
            raise ValueError("only backend: fake is available offline (COCO cannot be downloaded here)")
        model, self.criterion = detr.build(self.hp)
        self.model = context.wrap_model(model)
        self.criterion.to(context.device)
        print("number of params:", sum(p.numel() for p in model.parameters() if p.requires_grad))
        groups = [
            {"params": [p for n, p in self.model.named_parameters() if "backbone" not in n and p.requires_grad]},
            {"params": [p for n, p in self.model.named_parameters() if "backbone" in n and p.requires_grad],
             "lr": float(self.hp["lr_backbone"])},
        ]
        groups = [g for g in groups if g["params"]]
        self.optimizer = context.wrap_optimizer(torch.optim.AdamW(
            groups, lr=float(self.hp["lr"]), weight_decay=float(self.hp["weight_decay"])))
        self.lr_scheduler = context.wrap_lr_scheduler(
            torch.optim.lr_scheduler.StepLR(self.optimizer, int(self.hp["lr_drop"])),
            step_mode=pytorch.LRScheduler.StepMode.STEP_EVERY_EPOCH)
        amp = self.hp.get("amp")
        if amp and amp != "O0":
            self.model, self.optimizer = context.configure_apex_amp(self.model, self.optimizer, opt_level=amp)
        clip = float(self.hp.get("clip_max_norm", 0.0))
        self.clip_grads = pytorch.ClipGradsNorm(clip) if clip > 0 else None

    def _dataset(self, train: bool) -> SyntheticDetection:
        n = int(self.hp.get("train_records" if train else "validation_records", 117264 if train else 5000))
        return SyntheticDetection(n, num_classes=91, min_size=int(self.hp.get("min_image_size", 480)),
                                  max_size=int(self.hp.get("max_image_size", 640)), seed=0 if train else 1)

    @property
    def _collate(self):
        # padded shapes bucketed to 128 px (masked padding; few distinct conv shapes for MIOpen)
        return functools.partial(pad_collate, multiple=int(self.hp.get("pad_multiple", 128)))

    def build_training_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(self._dataset(True), batch_size=self.context.get_per_slot_batch_size(),
                                  collate_fn=self._collate, shuffle=True,
                                  num_workers=int(self.hp.get("num_workers", 0)))

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(self._dataset(False), batch_size=self.context.get_per_slot_batch_size(),
                                  collate_fn=self._collate, shuffle=False,
                                  num_workers=int(self.hp.get("num_workers", 0)))

    def _losses(self, outputs: Dict[str, Any], targets: Any, eval: bool = False) -> Dict[str, torch.Tensor]:
        loss_dict = self.criterion(outputs, targets, eval=eval)
        w = self.criterion.weight_dict
        scaled = {f"{k}_scaled": v * w[k] for k, v in loss_dict.items() if k in w}
        loss_dict["sum_unscaled"] = sum(loss_dict.values())
        loss_dict["sum_scaled"] = sum(scaled.values())
        loss_dict.update(scaled)
        return loss_dict

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        samples, targets = batch
        outputs = self.model(samples)
        loss_dict = self.criterion(outputs, targets)
        w = self.criterion.weight_dict
        loss = sum(loss_dict[k] * w[k] for k in loss_dict if k in w)
        self.context.backward(loss)
        self.context.step_optimizer(self.optimizer, clip_grads=self.clip_grads)
        scaled = {f"{k}_scaled": v * w[k] for k, v in loss_dict.items() if k in w}
        out = {k: v.detach() for k, v in loss_dict.items()}
        out["sum_unscaled"] = sum(out.values())
        out["sum_scaled"] = sum(v.detach() for v in scaled.values())
        out.update({k: v.detach() for k, v in scaled.items()})
        out["loss"] = loss.detach()
        return out

    def evaluate_full_dataset(self, data_loader: torch.utils.data.DataLoader) -> Dict[str, Any]:
        evaluator = CocoBboxEvaluator()
        agg: Dict[str, float] = defaultdict(float)
        n = 0
        with torch.no_grad():
            for batch in data_loader:
                samples, targets = self.context.to_device(batch)
                outputs = self.model(samples)
                for k, v in self._losses(outputs, targets, eval=True).items():
                    agg[k] += float(v)
                n += 1
                sizes = torch.stack([t["orig_size"] for t in targets])
                for t, res in zip(targets, postprocess(outputs, sizes)):
                    h, w = t["orig_size"].tolist()
                    gt = box_cxcywh_to_xyxy(t["boxes"].float()) * torch.tensor([w, h, w, h], device=t["boxes"].device)
                    evaluator.add(int(t["image_id"].item()), res, gt, t["labels"])
        metrics = {k: v / max(n, 1) for k, v in agg.items()}
        stats = evaluator.summarize()
        for name, v in zip(("mAP", "mAP_50", "mAP_75", "mAP_small", "mAP_medium", "mAP_large"), stats):
            metrics[name] = v
        return metrics
