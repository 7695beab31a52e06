"""Mask R-CNN R50-FPN (He et al. 2017) on the torchvision-free Faster R-CNN of ``faster_rcnn.py``:
the reference trains it through mmdetection (``examples/computer_vision/mmdetection_pytorch/
maskrcnn.yaml``; 0.310 s/iter on 8xV100 at 2 images per GPU, README.md:21,44), which is not in this
image, so the model family is rebuilt here on the same MI355X detection ops.

MI355X-specific choices:
  * mask RoI features (14x14 over P2-P5) and the mask targets (28x28 crops of the instance masks)
    both come from the NHWC multi-level ``det_roi_align`` HIP kernel -- the gt masks of a batch are
    one [N, H, W, G] "feature map", each positive RoI pools its matched instance's channel;
  * the mask-head batch (positive RoIs of the whole batch) is padded to a multiple of
    ``mask_bucket`` (zero-weighted dummy RoIs), so the head's convolutions see a handful of shapes and
    MIOpen never re-runs find mid-training (the same reason the image batch is bucketed).
"""
import math
from typing import List, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_1_amd.models.faster_rcnn import FasterRCNN, RoIHeads
from determined_1_amd.ops import detect


class MaskHead(nn.Module):
    """4 x (3x3 conv 256 + ReLU) -> 2x2/2 transposed conv + ReLU -> 1x1 conv to per-class logits."""

    def __init__(self, c: int, num_classes: int, width: int = 256, layers: int = 4) -> None:
        super().__init__()
        convs = []
        for i in range(layers):
            convs += [nn.Conv2d(c if i == 0 else width, width, 3, padding=1), nn.ReLU(inplace=True)]
        self.convs = nn.Sequential(*convs)
        self.deconv = nn.ConvTranspose2d(width, width, 2, stride=2)
        self.logits = nn.Conv2d(width, num_classes, 1)
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                nn.init.zeros_(m.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.logits(F.relu(self.deconv(self.convs(x))))


class MaskRoIHeads(RoIHeads):
    def __init__(self, c: int, num_classes: int, mask_bucket: int = 64, **kw) -> None:
        super().__init__(c, num_classes, **kw)
        self.mask_head = MaskHead(c, num_classes)
        self.mask_bucket = max(1, int(mask_bucket))

    def _mask_logits(self, feats: List[torch.Tensor], rois: torch.Tensor, image_hw: Tuple[int, int]) -> torch.Tensor:
        maps = feats[:4]
        scales = [2.0 ** round(math.log2(f.shape[-2] / image_hw[0])) for f in maps]
        k_min, k_max = int(-math.log2(scales[0])), int(-math.log2(scales[-1]))
        levels = detect.map_levels(rois[:, 1:], k_min, k_max)
        x = detect.roi_align_multilevel(maps, rois, levels, scales, 14, 2)  # [P, 14, 14, C]
        x = x.permute(0, 3, 1, 2)  # NCHW view of the NHWC result (channels_last)
        return self.mask_head(x)

    def forward(self, feats, proposals, image_hw, sizes, targets=None):
        results, losses = super().forward(feats, proposals, image_hw, sizes, targets)
        if self.training:
            losses["loss_mask"] = self._mask_loss(feats, image_hw, targets)
            return results, losses
        boxes = [r["boxes"] for r in results]
        rois = torch.cat([torch.cat([torch.full((b.shape[0], 1), float(i), device=b.device), b.float()], 1)
                          for i, b in enumerate(boxes)])
        if rois.shape[0]:
            prob = self._mask_logits(feats, rois, image_hw).float().sigmoid()
            lab = torch.cat([r["labels"] for r in results])
            prob = prob[torch.arange(prob.shape[0], device=prob.device), lab]
        else:
            prob = feats[0].new_zeros((0, 28, 28), dtype=torch.float32)
        for r, m in zip(results, prob.split([b.shape[0] for b in boxes])):
            r["masks"] = m
        return results, losses

    def _mask_loss(self, feats, image_hw, targets) -> torch.Tensor:
        props, labs, mids = self.sampled
        dev = feats[0].device
        rois, lab_p, gid = [], [], []
        for i, (p, lab, mid) in enumerate(zip(props, labs, mids)):
            pos = torch.nonzero(lab > 0).flatten()
            rois.append(torch.cat([torch.full((pos.numel(), 1), float(i), device=dev), p[pos].float()], 1))
            lab_p.append(lab[pos])
            gid.append(mid[pos])
        rois, lab_p, gid = torch.cat(rois), torch.cat(lab_p), torch.cat(gid)
        n = rois.shape[0]
        if n == 0:
            return sum(p.sum() for p in self.mask_head.parameters()) * 0.0
        padded = (n + self.mask_bucket - 1) // self.mask_bucket * self.mask_bucket
        if padded > n:  # zero-weighted dummy RoIs: the head's conv batch takes few distinct sizes
            dummy = torch.tensor([[0.0, 0.0, 0.0, 16.0, 16.0]], device=dev).expand(padded - n, 5)
            rois_all = torch.cat([rois, dummy])
        else:
            rois_all = rois
        logits = self._mask_logits(feats, rois_all, image_hw)[:n]
        logits = logits[torch.arange(n, device=dev), lab_p]  # [n, 28, 28]
        tgt = self._mask_targets(targets, rois, gid, image_hw, logits.shape[-1])
        return F.binary_cross_entropy_with_logits(logits.float(), tgt)

    @staticmethod
    def _mask_targets(targets, rois, gid, image_hw, size: int) -> torch.Tensor:
        """28x28 crops of each positive RoI's matched instance mask (RoIAlign over the stacked masks)."""
        g = max(int(t["masks"].shape[0]) for t in targets)
        g8 = max(8, (g + 7) // 8 * 8)
        h, w = image_hw
        dev = rois.device
        dt = torch.bfloat16 if dev.type == "cuda" else torch.float32
        stack = torch.zeros((len(targets), h, w, g8), dtype=dt, device=dev)
        for i, t in enumerate(targets):
            mk = t["masks"]
            if mk.numel():
                stack[i, :mk.shape[1], :mk.shape[2], :mk.shape[0]] = mk.to(device=dev, dtype=dt).permute(1, 2, 0)
        levels = torch.zeros(rois.shape[0], dtype=torch.int64, device=dev)
        crops = detect.roi_align_multilevel([stack.permute(0, 3, 1, 2)], rois, levels, [1.0], size, 2)
        sel = crops[torch.arange(rois.shape[0], device=dev), :, :, gid]  # [n, size, size]
        return (sel.float() >= 0.5).float()


class MaskRCNN(FasterRCNN):
    """Faster R-CNN + a mask branch; ``forward`` returns the losses (incl. ``loss_mask``) in training
    and per-image ``boxes``/``scores``/``labels``/``masks`` (``[D, 1, H, W]`` probabilities) in eval."""

    def __init__(self, num_classes: int = 91, mask_bucket: int = 64, **kw) -> None:
        self._mask_bucket = mask_bucket
        super().__init__(num_classes=num_classes, **kw)

    def _make_roi_heads(self, c: int, num_classes: int) -> RoIHeads:
        return MaskRoIHeads(c, num_classes, mask_bucket=self._mask_bucket)


def maskrcnn_resnet50_fpn(num_classes: int = 91, **kw) -> MaskRCNN:
    return MaskRCNN(num_classes=num_classes, arch="resnet50", **kw)


__all__ = ["MaskHead", "MaskRoIHeads", "MaskRCNN", "maskrcnn_resnet50_fpn"]
