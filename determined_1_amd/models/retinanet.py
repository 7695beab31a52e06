"""RetinaNet R50-FPN (Lin et al. 2017), the one-stage member of the detection family the reference
trains through mmdetection (``examples/computer_vision/mmdetection_pytorch/retinanet.yaml`` ->
``retinanet_r50_fpn_1x_coco``).  mmdetection is not in this image; the model is built on the
torchvision-free pieces of ``faster_rcnn.py`` (frozen-BN ResNet body, anchors, box coder, matcher,
transform) and the MI355X detection ops (device NMS).

Layout: P3-P7 pyramid (P6 = 3x3/2 conv on P5, P7 = 3x3/2 conv on relu(P6)), 9 anchors per
location (3 octave scales x 3 ratios), 4-conv classification and box subnets shared across levels,
sigmoid focal loss (alpha 0.25, gamma 2) and L1 box loss normalised by the foreground count.
"""
import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_1_amd.models.detr import BACKBONE_LAYERS, FrozenBNResNet
from determined_1_amd.models.faster_rcnn import (BELOW, BETWEEN, AnchorGenerator, BoxCoder, ImageBatchTransform,
                                                 box_iou, match)
from determined_1_amd.ops import conv as native_conv
from determined_1_amd.ops import detect



class _NativeConv(nn.Conv2d):
    """An ``nn.Conv2d`` whose forward runs on the native kernels where they cover the shape (the
    256-channel head towers); same parameters and state dict as the module it replaces."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        return native_conv.conv2d_module(x, self, fallback=super().forward)

class RetinaFPN(nn.Module):
    def __init__(self, arch: str = "resnet50", trainable_layers: int = 3, out: int = 256) -> None:
        super().__init__()
        self.body = FrozenBNResNet(BACKBONE_LAYERS[arch], train_backbone=True)
        trainable = ["layer4", "layer3", "layer2", "layer1", "stem"][:trainable_layers]
        for name, p in self.body.named_parameters():
            p.requires_grad_(any(name.startswith(t) for t in trainable))
        self.inner = nn.ModuleList(nn.Conv2d(c, out, 1) for c in (512, 1024, 2048))
        self.layer = nn.ModuleList(nn.Conv2d(out, out, 3, padding=1) for _ in range(3))
        self.p6 = nn.Conv2d(out, out, 3, stride=2, padding=1)
        self.p7 = nn.Conv2d(out, out, 3, stride=2, padding=1)
        for m in [*self.inner, *self.layer, self.p6, self.p7]:
            nn.init.kaiming_uniform_(m.weight, a=1)
            nn.init.constant_(m.bias, 0)
        self.out_channels = out

    def forward(self, x: torch.Tensor) -> List[torch.Tensor]:
        b = self.body
        c = F.max_pool2d(F.relu(b.stem(x), inplace=True), 3, 2, 1)
        c3 = b.layer2(b.layer1(c))
        c4 = b.layer3(c3)
        c5 = b.layer4(c4)
        cm = native_conv.conv2d_module  # FPN convs on the native kernels
        last = cm(c5, self.inner[2])
        outs = [cm(last, self.layer[2])]
        for i, ci in ((1, c4), (0, c3)):
            lat = cm(ci, self.inner[i])
            last = lat + F.interpolate(last, size=lat.shape[-2:], mode="nearest")
            outs.insert(0, cm(last, self.layer[i]))
        p6 = cm(outs[-1], self.p6)
        return outs + [p6, cm(F.relu(p6), self.p7)]


class RetinaAnchors(AnchorGenerator):
    """3 octave scales x 3 aspect ratios per level (anchor sizes 32..512 on P3..P7)."""

    def __init__(self, sizes: Sequence[int] = (32, 64, 128, 256, 512), ratios: Sequence[float] = (0.5, 1.0, 2.0),
                 octaves: Sequence[float] = (1.0, 2 ** (1 / 3), 2 ** (2 / 3))) -> None:
        super().__init__(sizes, ratios)
        self.octaves = octaves

    def num_anchors(self) -> int:
        return len(self.ratios) * len(self.octaves)

    def _base(self, size: int, device: torch.device) -> torch.Tensor:
        r = torch.tensor(self.ratios, dtype=torch.float32, device=device)
        s = torch.tensor(self.octaves, dtype=torch.float32, device=device) * size
        h_ratio = r.sqrt()
        w_ratio = 1 / h_ratio
        ws = (w_ratio[:, None] * s[None]).reshape(-1)
        hs = (h_ratio[:, None] * s[None]).reshape(-1)
        return (torch.stack([-ws, -hs, ws, hs], 1) / 2).round()


class RetinaHead(nn.Module):
    def __init__(self, c: int, a: int, num_classes: int, convs: int = 4, prior: float = 0.01) -> None:
        super().__init__()

        def tower():
            layers = []
            for _ in range(convs):
                layers += [_NativeConv(c, c, 3, padding=1), nn.ReLU(inplace=True)]
            return nn.Sequential(*layers)

        self.cls_tower, self.box_tower = tower(), tower()
        self.cls_logits = nn.Conv2d(c, a * num_classes, 3, padding=1)
        self.bbox_pred = nn.Conv2d(c, a * 4, 3, padding=1)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.normal_(m.weight, std=0.01)
                nn.init.constant_(m.bias, 0)
        nn.init.constant_(self.cls_logits.bias, -math.log((1 - prior) / prior))
        self.a, self.k = a, num_classes

    def forward(self, feats: List[torch.Tensor]) -> Tuple[List[torch.Tensor], List[torch.Tensor]]:
        """-> per level ``[N, H*W*A, K]`` class logits and ``[N, H*W*A, 4]`` deltas (anchor-minor)."""
        cls, box = [], []
        for f in feats:
            c, d = self.cls_logits(self.cls_tower(f)), self.bbox_pred(self.box_tower(f))
            n, _, h, w = c.shape
            cls.append(c.view(n, self.a, self.k, h, w).permute(0, 3, 4, 1, 2).reshape(n, -1, self.k))
            box.append(d.view(n, self.a, 4, h, w).permute(0, 3, 4, 1, 2).reshape(n, -1, 4))
        return cls, box


def sigmoid_focal_loss(logits: torch.Tensor, targets: torch.Tensor, alpha: float = 0.25, gamma: float = 2.0) -> torch.Tensor:
    p = logits.sigmoid()
    ce = F.binary_cross_entropy_with_logits(logits, targets, reduction="none")
    p_t = p * targets + (1 - p) * (1 - targets)
    loss = ce * (1 - p_t) ** gamma
    return (alpha * targets + (1 - alpha) * (1 - targets)) * loss


class RetinaNet(ImageBatchTransform):
    """``forward(images, targets)`` -> ``{"classification", "bbox_regression"}`` losses in training,
    per-image ``boxes``/``scores``/``labels`` in eval.  Same resize/normalise/pad transform as the
    two-stage detectors (``size_divisible`` buckets the padded batch shape)."""

    def __init__(self, num_classes: int = 91, min_size: int = 800, max_size: int = 1333, arch: str = "resnet50",
                 trainable_layers: int = 3, channels_last: bool = True, size_divisible: int = 128,
                 score_thresh: float = 0.05, nms_thresh: float = 0.5, detections_per_img: int = 100,
                 topk_candidates: int = 1000, fg_iou: float = 0.5, bg_iou: float = 0.4) -> None:
        super().__init__(min_size, max_size, size_divisible, channels_last)
        self.backbone = RetinaFPN(arch, trainable_layers)
        self.anchors = RetinaAnchors()
        self.head = RetinaHead(self.backbone.out_channels, self.anchors.num_anchors(), num_classes)
        self.coder = BoxCoder((1.0, 1.0, 1.0, 1.0))
        self.num_classes = num_classes
        self.score_thresh, self.nms_thresh, self.detections_per_img = score_thresh, nms_thresh, detections_per_img
        self.topk_candidates, self.fg_iou, self.bg_iou = topk_candidates, fg_iou, bg_iou

    def forward(self, images: Sequence[torch.Tensor], targets: Optional[List[Dict[str, torch.Tensor]]] = None):
        if self.training and targets is None:
            raise ValueError("targets are required in training mode")
        orig = [tuple(img.shape[-2:]) for img in images]
        batch, sizes, targets = self._transform(images, targets)
        feats = self.backbone(batch)
        image_hw = (batch.shape[-2], batch.shape[-1])
        cls, box = self.head(feats)
        anchors = self.anchors(image_hw, feats)
        if self.training:
            return self._losses(torch.cat(cls, 1), torch.cat(box, 1), anchors, targets)
        dets = self._detections(cls, box, anchors, sizes)
        for d, s, o in zip(dets, sizes, orig):
            ry, rx = o[0] / s[0], o[1] / s[1]
            d["boxes"] = d["boxes"] * torch.tensor([rx, ry, rx, ry], device=d["boxes"].device)
        return dets

    def _losses(self, cls, box, anchors, targets) -> Dict[str, torch.Tensor]:
        cls_l, box_l, n_fg = [], [], 0
        for i, t in enumerate(targets):
            gt, gl = t["boxes"].float(), t["labels"]
            tgt = torch.zeros_like(cls[i], dtype=torch.float32)
            if gt.numel():
                m = match(box_iou(gt, anchors), self.fg_iou, self.bg_iou, allow_low_quality=True)
            else:
                m = torch.full((anchors.shape[0],), BELOW, dtype=torch.int64, device=anchors.device)
            fg = torch.nonzero(m >= 0).flatten()
            valid = m != BETWEEN
            if fg.numel():
                tgt[fg, gl[m[fg]]] = 1.0
                box_l.append(F.l1_loss(box[i, fg].float(), self.coder.encode(gt[m[fg]], anchors[fg]), reduction="sum"))
            cls_l.append(sigmoid_focal_loss(cls[i][valid].float(), tgt[valid]).sum())
            n_fg += int(fg.numel())
        norm = max(1.0, float(n_fg))
        zero = box.sum() * 0.0
        return {"classification": sum(cls_l) / norm, "bbox_regression": (sum(box_l) if box_l else zero) / norm}

    def _detections(self, cls, box, anchors, sizes) -> List[Dict[str, torch.Tensor]]:
        counts = [c.shape[1] for c in cls]
        anchors_l = anchors.split(counts)
        out = []
        for i, size in enumerate(sizes):
            bs, ss, ls = [], [], []
            for c, d, a in zip(cls, box, anchors_l):
                sc = c[i].float().sigmoid().flatten()
                keep = torch.nonzero(sc > self.score_thresh).flatten()
                sc = sc[keep]
                if sc.numel() > self.topk_candidates:
                    sc, top = sc.topk(self.topk_candidates)
                    keep = keep[top]
                if keep.numel() == 0:
                    continue
                aidx, lab = keep // self.num_classes, keep % self.num_classes
                b = self.coder.decode(d[i, aidx].float(), a[aidx]).reshape(-1, 4)
                bs.append(detect.clip_boxes_to_image(b, list(size)))
                ss.append(sc)
                ls.append(lab)
            if not bs:
                dev = anchors.device
                out.append({"boxes": torch.zeros((0, 4), device=dev), "scores": torch.zeros((0,), device=dev),
                            "labels": torch.zeros((0,), dtype=torch.int64, device=dev)})
                continue
            b, s, lab = torch.cat(bs), torch.cat(ss), torch.cat(ls)
            keep = detect.batched_nms(b, s, lab, self.nms_thresh)[:self.detections_per_img]
            out.append({"boxes": b[keep], "scores": s[keep], "labels": lab[keep]})
        return out


def retinanet_resnet50_fpn(num_classes: int = 91, **kw) -> RetinaNet:
    return RetinaNet(num_classes=num_classes, arch="resnet50", **kw)


__all__ = ["RetinaFPN", "RetinaAnchors", "RetinaHead", "RetinaNet", "retinanet_resnet50_fpn", "sigmoid_focal_loss"]
