"""Faster R-CNN with a ResNet-50-FPN backbone (Ren et al. 2015; Lin et al. 2017) -- the model the
reference's detection example builds with ``torchvision.models.detection.fasterrcnn_resnet50_fpn``
and a 2-class ``FastRCNNPredictor`` (``examples/computer_vision/fasterrcnn_coco_pytorch/
model_def.py:48-53``).  torchvision is not in this image; this is a from-scratch implementation
with torchvision's default hyper-parameters and training semantics:

  transform  normalise (ImageNet mean/std), resize shorter side to 800 (longer <= 1333), pad the
             batch to a multiple of 32; detections are mapped back to the original image size;
  backbone   ResNet-50 with frozen BatchNorm (folded into the convs, ``detr.FrozenBNResNet``), only
             layer2-4 trainable, + FPN (256 channels, P2-P5 and a max-pooled P6);
  RPN        3 anchors per location and level (sizes 32..512, ratios 0.5/1/2), shared 3x3 head,
             IoU matching 0.7/0.3 with low-quality matches, 256 samples/image at 50 % positives,
             top-2000 (train) / 1000 (test) per level before NMS 0.7, 2000 / 1000 after;
  RoI heads  multi-level RoIAlign 7x7 (sampling 2), two 1024-wide FC layers, class + class-specific
             box predictor, matching 0.5, 512 samples/image at 25 % positives, box coder weights
             (10, 10, 5, 5), smooth-L1 beta 1/9; inference: score > 0.05, per-class NMS 0.5, <= 100
             detections.

MI355X-specific execution: feature maps stay channels_last end to end; RoIAlign for all four FPN
levels is ONE launch of the NHWC ``det_roi_align`` HIP kernel (fwd and bwd), and every NMS --
RPN proposals per image and per-class detections -- runs on the device (``det_nms``: 64x64-tile
IoU bitmask + single-wave sweep), so the proposal path never round-trips boxes through the host.
Anchors are generated once per feature-map geometry and cached on the device.
"""
import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_1_amd.models.detr import BACKBONE_LAYERS, FrozenBNResNet
from determined_1_amd.ops import conv as native_conv
from determined_1_amd.ops import detect

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


# ------------------------------------------------------------------------------------------------
# box coding, matching, sampling
# ------------------------------------------------------------------------------------------------
class BoxCoder:
    def __init__(self, weights: Tuple[float, float, float, float], clip: float = math.log(1000.0 / 16)) -> None:
        self.weights, self.clip = weights, clip

    def encode(self, gt: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
        wx, wy, ww, wh = self.weights
        rw, rh = ref[:, 2] - ref[:, 0], ref[:, 3] - ref[:, 1]
        rx, ry = ref[:, 0] + 0.5 * rw, ref[:, 1] + 0.5 * rh
        gw, gh = gt[:, 2] - gt[:, 0], gt[:, 3] - gt[:, 1]
        gx, gy = gt[:, 0] + 0.5 * gw, gt[:, 1] + 0.5 * gh
        return torch.stack([wx * (gx - rx) / rw, wy * (gy - ry) / rh, ww * torch.log(gw / rw), wh * torch.log(gh / rh)], 1)

    def decode(self, codes: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
        """``codes [N, 4k]`` relative to ``ref [N, 4]`` -> boxes ``[N, k, 4]``."""
        ref = ref.to(codes.dtype)
        wx, wy, ww, wh = self.weights
        w, h = ref[:, 2] - ref[:, 0], ref[:, 3] - ref[:, 1]
        cx, cy = ref[:, 0] + 0.5 * w, ref[:, 1] + 0.5 * h
        c = codes.reshape(codes.shape[0], -1, 4)
        dx, dy = c[..., 0] / wx, c[..., 1] / wy
        dw, dh = (c[..., 2] / ww).clamp(max=self.clip), (c[..., 3] / wh).clamp(max=self.clip)
        px, py = dx * w[:, None] + cx[:, None], dy * h[:, None] + cy[:, None]
        pw, ph = torch.exp(dw) * w[:, None], torch.exp(dh) * h[:, None]
        return torch.stack([px - 0.5 * pw, py - 0.5 * ph, px + 0.5 * pw, py + 0.5 * ph], -1)


BELOW, BETWEEN = -1, -2


def match(iou: torch.Tensor, high: float, low: float, allow_low_quality: bool) -> torch.Tensor:
    """``iou [G, P]`` -> matched gt index per prediction, ``BELOW`` / ``BETWEEN`` otherwise."""
    if iou.shape[0] == 0:
        return torch.full((iou.shape[1],), BELOW, dtype=torch.int64, device=iou.device)
    vals, idx = iou.max(0)
    all_idx = idx.clone()
    idx[vals < low] = BELOW
    idx[(vals >= low) & (vals < high)] = BETWEEN
    if allow_low_quality:  # keep, for every gt, the predictions that overlap it best
        best = iou.max(1).values
        pred = torch.nonzero(iou == best[:, None])[:, 1]
        idx[pred] = all_idx[pred]
    return idx


def sample(labels: torch.Tensor, per_image: int, pos_fraction: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """Balanced random subset: returns (positive indices, negative indices)."""
    pos = torch.nonzero(labels >= 1).flatten()
    neg = torch.nonzero(labels == 0).flatten()
    n_pos = min(int(per_image * pos_fraction), pos.numel())
    n_neg = min(per_image - n_pos, neg.numel())
    pos = pos[torch.randperm(pos.numel(), device=pos.device)[:n_pos]]
    neg = neg[torch.randperm(neg.numel(), device=neg.device)[:n_neg]]
    return pos, neg


def box_iou(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return detect.pairwise_iou(a, b)


# ------------------------------------------------------------------------------------------------
# backbone + FPN
# ------------------------------------------------------------------------------------------------
class FPN(nn.Module):
    def __init__(self, in_channels: Sequence[int], out: int = 256) -> None:
        super().__init__()
        self.inner = nn.ModuleList(nn.Conv2d(c, out, 1) for c in in_channels)
        self.layer = nn.ModuleList(nn.Conv2d(out, out, 3, padding=1) for _ in in_channels)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_uniform_(m.weight, a=1)
                nn.init.constant_(m.bias, 0)

    def forward(self, xs: List[torch.Tensor]) -> List[torch.Tensor]:
        cm = native_conv.conv2d_module  # the 1x1 laterals and 3x3 outputs on the native kernels
        last = cm(xs[-1], self.inner[-1])
        outs = [cm(last, self.layer[-1])]
        for i in range(len(xs) - 2, -1, -1):
            lateral = cm(xs[i], self.inner[i])
            last = lateral + F.interpolate(last, size=lateral.shape[-2:], mode="nearest")
            outs.insert(0, cm(last, self.layer[i]))
        outs.append(F.max_pool2d(outs[-1], 1, 2, 0))  # P6 (LastLevelMaxPool)
        return outs


class ResNetFPN(nn.Module):
    def __init__(self, arch: str = "resnet50", trainable_layers: int = 3) -> None:
        super().__init__()
        self.body = FrozenBNResNet(BACKBONE_LAYERS[arch], train_backbone=True)
        trainable = ["layer4", "layer3", "layer2", "layer1", "stem"][:trainable_layers]
        for name, p in self.body.named_parameters():
            p.requires_grad_(any(name.startswith(t) for t in trainable))
        self.fpn = FPN([256, 512, 1024, 2048], 256)
        self.out_channels = 256

    def forward(self, x: torch.Tensor) -> List[torch.Tensor]:
        b = self.body
        c1 = F.max_pool2d(F.relu(b.stem(x), inplace=True), 3, 2, 1)
        c2 = b.layer1(c1)
        c3 = b.layer2(c2)
        c4 = b.layer3(c3)
        c5 = b.layer4(c4)
        return self.fpn([c2, c3, c4, c5])


# ------------------------------------------------------------------------------------------------
# RPN
# ------------------------------------------------------------------------------------------------
class AnchorGenerator:
    def __init__(self, sizes: Sequence[int] = (32, 64, 128, 256, 512), ratios: Sequence[float] = (0.5, 1.0, 2.0)) -> None:
        self.sizes, self.ratios = sizes, ratios
        self._cache: Dict[Tuple, torch.Tensor] = {}

    def num_anchors(self) -> int:
        return len(self.ratios)

    def _base(self, size: int, device: torch.device) -> torch.Tensor:
        r = torch.tensor(self.ratios, dtype=torch.float32, device=device)
        h_ratio = r.sqrt()
        w_ratio = 1 / h_ratio
        ws, hs = w_ratio * size, h_ratio * size
        return (torch.stack([-ws, -hs, ws, hs], 1) / 2).round()

    def __call__(self, image_hw: Tuple[int, int], feats: List[torch.Tensor]) -> torch.Tensor:
        """Anchors of all levels for one padded batch geometry: ``[sum_l H_l*W_l*A, 4]``."""
        key = (image_hw, tuple(tuple(f.shape[-2:]) for f in feats), feats[0].device)
        hit = self._cache.get(key)
        if hit is not None:
            return hit
        out = []
        for f, size in zip(feats, self.sizes):
            h, w = f.shape[-2:]
            sy, sx = image_hw[0] // h, image_hw[1] // w
            ys = torch.arange(h, dtype=torch.float32, device=f.device) * sy
            xs = torch.arange(w, dtype=torch.float32, device=f.device) * sx
            yy, xx = torch.meshgrid(ys, xs, indexing="ij")
            shifts = torch.stack([xx.reshape(-1), yy.reshape(-1), xx.reshape(-1), yy.reshape(-1)], 1)
            out.append((shifts[:, None, :] + self._base(size, f.device)[None]).reshape(-1, 4))
        anchors = torch.cat(out)
        if len(self._cache) > 16:
            self._cache.clear()
        self._cache[key] = anchors
        return anchors


class RPNHead(nn.Module):
    def __init__(self, c: int, a: int) -> None:
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, padding=1)
        self.cls_logits = nn.Conv2d(c, a, 1)
        self.bbox_pred = nn.Conv2d(c, 4 * a, 1)
        for m in (self.conv, self.cls_logits, self.bbox_pred):
            nn.init.normal_(m.weight, std=0.01)
            nn.init.constant_(m.bias, 0)

    def forward(self, feats: List[torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor, List[int]]:
        """-> objectness ``[N, sum HWA]``, deltas ``[N, sum HWA, 4]``, anchors per level."""
        objs, deltas, counts = [], [], []
        for f in feats:
            t = F.relu(native_conv.conv2d_module(f, self.conv))
            o, d = self.cls_logits(t), self.bbox_pred(t)
            n, a, h, w = o.shape
            objs.append(o.permute(0, 2, 3, 1).reshape(n, -1))  # location-major, anchor-minor
            deltas.append(d.view(n, a, 4, h, w).permute(0, 3, 4, 1, 2).reshape(n, -1, 4))
            counts.append(h * w * a)
        return torch.cat(objs, 1), torch.cat(deltas, 1), counts


def smooth_l1(x: torch.Tensor, y: torch.Tensor, beta: float) -> torch.Tensor:
    d = (x - y).abs()
    return torch.where(d < beta, 0.5 * d * d / beta, d - 0.5 * beta).sum()


class RPN(nn.Module):
    def __init__(self, c: int, pre_nms: Dict[str, int], post_nms: Dict[str, int], nms_thresh: float = 0.7,
                 fg_iou: float = 0.7, bg_iou: float = 0.3, per_image: int = 256, pos_fraction: float = 0.5) -> None:
        super().__init__()
        self.anchors = AnchorGenerator()
        self.head = RPNHead(c, self.anchors.num_anchors())
        self.coder = BoxCoder((1.0, 1.0, 1.0, 1.0))
        self.pre_nms, self.post_nms, self.nms_thresh = pre_nms, post_nms, nms_thresh
        self.fg_iou, self.bg_iou, self.per_image, self.pos_fraction = fg_iou, bg_iou, per_image, pos_fraction

    def _proposals(self, obj: torch.Tensor, boxes: torch.Tensor, counts: List[int], sizes: List[Tuple[int, int]]
                   ) -> List[torch.Tensor]:
        mode = "training" if self.training else "testing"
        k_pre, k_post = self.pre_nms[mode], self.post_nms[mode]
        n = obj.shape[0]
        # top-k per level (all images at once), level id per kept candidate
        sel, lvl = [], []
        off = 0
        for li, cnt in enumerate(counts):
            k = min(k_pre, cnt)
            _, idx = obj[:, off:off + cnt].topk(k, dim=1)
            sel.append(idx + off)
            lvl.append(torch.full((k,), li, dtype=torch.int64, device=obj.device))
            off += cnt
        sel_t = torch.cat(sel, 1)
        lvl_t = torch.cat(lvl)
        bidx = torch.arange(n, device=obj.device)[:, None]
        scores = obj[bidx, sel_t].sigmoid()
        cand = boxes[bidx, sel_t]
        out = []
        for i in range(n):
            b = detect.clip_boxes_to_image(cand[i], list(sizes[i]))
            keep = detect.remove_small_boxes(b, 1e-3)
            b, s, lv = b[keep], scores[i][keep], lvl_t[keep]
            keep = detect.batched_nms(b, s, lv, self.nms_thresh)[:k_post]
            out.append(b[keep])
        return out

    def forward(self, feats: List[torch.Tensor], image_hw: Tuple[int, int], sizes: List[Tuple[int, int]],
                targets: Optional[List[Dict[str, torch.Tensor]]] = None) -> Tuple[List[torch.Tensor], Dict[str, torch.Tensor]]:
        obj, deltas, counts = self.head(feats)
        anchors = self.anchors(image_hw, feats)
        n = obj.shape[0]
        with torch.no_grad():
            boxes = self.coder.decode(deltas.detach().reshape(-1, 4).float(), anchors.repeat(n, 1)).view(n, -1, 4)
            proposals = self._proposals(obj.detach().float(), boxes, counts, sizes)
        losses: Dict[str, torch.Tensor] = {}
        if self.training:
            assert targets is not None
            pos_all, neg_all, tgt_all = [], [], []
            for i, t in enumerate(targets):
                gt = t["boxes"]
                m = match(box_iou(gt, anchors), self.fg_iou, self.bg_iou, allow_low_quality=True)
                labels = (m >= 0).to(torch.float32)
                labels[m == BETWEEN] = -1.0
                pos, neg = sample(labels, self.per_image, self.pos_fraction)
                off = i * anchors.shape[0]
                pos_all.append(pos + off)
                neg_all.append(neg + off)
                if gt.numel():
                    tgt_all.append(self.coder.encode(gt[m[pos].clamp(min=0)], anchors[pos]))
                else:
                    tgt_all.append(anchors.new_zeros(0, 4))
            pos_t, neg_t = torch.cat(pos_all), torch.cat(neg_all)
            idx = torch.cat([pos_t, neg_t])
            lab = torch.cat([torch.ones_like(pos_t, dtype=torch.float32), torch.zeros_like(neg_t, dtype=torch.float32)])
            flat_obj = obj.reshape(-1).float()
            losses["loss_objectness"] = F.binary_cross_entropy_with_logits(flat_obj[idx], lab)
            losses["loss_rpn_box_reg"] = smooth_l1(deltas.reshape(-1, 4).float()[pos_t], torch.cat(tgt_all),
                                                   1.0 / 9) / max(idx.numel(), 1)
        return proposals, losses


# ------------------------------------------------------------------------------------------------
# RoI heads
# ------------------------------------------------------------------------------------------------
class RoIHeads(nn.Module):
    def __init__(self, c: int, num_classes: int, rep: int = 1024, fg_iou: float = 0.5, bg_iou: float = 0.5,
                 per_image: int = 512, pos_fraction: float = 0.25, score_thresh: float = 0.05, nms_thresh: float = 0.5,
                 detections_per_img: int = 100) -> None:
        super().__init__()
        self.fc6, self.fc7 = nn.Linear(c * 49, rep), nn.Linear(rep, rep)
        self.cls_score, self.bbox_pred = nn.Linear(rep, num_classes), nn.Linear(rep, num_classes * 4)
        self.coder = BoxCoder((10.0, 10.0, 5.0, 5.0))
        self.fg_iou, self.bg_iou, self.per_image, self.pos_fraction = fg_iou, bg_iou, per_image, pos_fraction
        self.score_thresh, self.nms_thresh, self.detections_per_img = score_thresh, nms_thresh, detections_per_img
        self.num_classes = num_classes

    def _pool(self, feats: List[torch.Tensor], proposals: List[torch.Tensor], image_hw: Tuple[int, int]) -> torch.Tensor:
        rois = torch.cat([torch.cat([torch.full((p.shape[0], 1), float(i), device=p.device), p.float()], 1)
                          for i, p in enumerate(proposals)])
        maps = feats[:4]  # P2-P5
        scales = [2.0 ** round(math.log2(f.shape[-2] / image_hw[0])) for f in maps]
        k_min, k_max = int(-math.log2(scales[0])), int(-math.log2(scales[-1]))
        levels = detect.map_levels(rois[:, 1:], k_min, k_max)
        return detect.roi_align_multilevel(maps, rois, levels, scales, 7, 2)

    def forward(self, feats: List[torch.Tensor], proposals: List[torch.Tensor], image_hw: Tuple[int, int],
                sizes: List[Tuple[int, int]], targets: Optional[List[Dict[str, torch.Tensor]]] = None
                ) -> Tuple[List[Dict[str, torch.Tensor]], Dict[str, torch.Tensor]]:
        labels_t = reg_t = None
        if self.training:
            assert targets is not None
            props, labs, regs, mids = [], [], [], []
            for p, t in zip(proposals, targets):
                gt, gl = t["boxes"].to(p.dtype), t["labels"]
                p = torch.cat([p, gt])
                if gt.numel():
                    m = match(box_iou(gt, p), self.fg_iou, self.bg_iou, allow_low_quality=False)
                    lab = gl[m.clamp(min=0)].to(torch.int64)
                    lab[m == BELOW] = 0
                    lab[m == BETWEEN] = -1
                    mg = gt[m.clamp(min=0)]
                else:
                    lab = torch.zeros(p.shape[0], dtype=torch.int64, device=p.device)
                    mg = torch.zeros_like(p)
                pos, neg = sample(lab, self.per_image, self.pos_fraction)
                keep = torch.cat([pos, neg])
                mid = m.clamp(min=0)[keep] if gt.numel() else torch.zeros_like(keep)
                p, lab, mg = p[keep], lab[keep], mg[keep]
                props.append(p)
                labs.append(lab)
                mids.append(mid)
                regs.append(self.coder.encode(mg, p))
            proposals = props
            labels_t, reg_t = torch.cat(labs), torch.cat(regs)
            self.sampled = (props, labs, mids)  # for heads that train on the same sample (masks)
        x = self._pool(feats, proposals, image_hw).flatten(1)
        x = F.relu(self.fc7(F.relu(self.fc6(x))))
        logits, box_reg = self.cls_score(x), self.bbox_pred(x)
        losses: Dict[str, torch.Tensor] = {}
        results: List[Dict[str, torch.Tensor]] = []
        if self.training:
            losses["loss_classifier"] = F.cross_entropy(logits.float(), labels_t)
            pos = torch.nonzero(labels_t > 0).flatten()
            reg = box_reg.float().view(box_reg.shape[0], -1, 4)[pos, labels_t[pos]]
            losses["loss_box_reg"] = smooth_l1(reg, reg_t[pos], 1.0 / 9) / max(labels_t.numel(), 1)
        else:
            results = self._detections(logits.float(), box_reg.float(), proposals, sizes)
        return results, losses

    def _detections(self, logits, box_reg, proposals, sizes) -> List[Dict[str, torch.Tensor]]:
        counts = [p.shape[0] for p in proposals]
        boxes = self.coder.decode(box_reg, torch.cat(proposals).float())
        scores = logits.softmax(-1)
        out = []
        for b, s, size in zip(boxes.split(counts), scores.split(counts), sizes):
            b = detect.clip_boxes_to_image(b, list(size))
            lab = torch.arange(self.num_classes, device=b.device).view(1, -1).expand_as(s)
            b, s, lab = b[:, 1:].reshape(-1, 4), s[:, 1:].reshape(-1), lab[:, 1:].reshape(-1)
            keep = torch.nonzero(s > self.score_thresh).flatten()
            b, s, lab = b[keep], s[keep], lab[keep]
            keep = detect.remove_small_boxes(b, 1e-2)
            b, s, lab = b[keep], s[keep], lab[keep]
            keep = detect.batched_nms(b, s, lab, self.nms_thresh)[:self.detections_per_img]
            out.append({"boxes": b[keep], "scores": s[keep], "labels": lab[keep]})
        return out


def paste_masks(masks: torch.Tensor, boxes: torch.Tensor, image_hw: Tuple[int, int]) -> torch.Tensor:
    """``masks [D, M, M]`` (probabilities over each box) -> ``[D, 1, H, W]`` full-image masks."""
    h, w = int(image_hw[0]), int(image_hw[1])
    out = masks.new_zeros((masks.shape[0], 1, h, w))
    for i in range(masks.shape[0]):
        x0, y0, x1, y1 = boxes[i].tolist()
        x0, y0 = max(int(math.floor(x0)), 0), max(int(math.floor(y0)), 0)
        x1, y1 = min(int(math.ceil(x1)), w), min(int(math.ceil(y1)), h)
        if x1 > x0 and y1 > y0:
            out[i, 0, y0:y1, x0:x1] = F.interpolate(masks[i][None, None], size=(y1 - y0, x1 - x0), mode="bilinear",
                                                    align_corners=False)[0, 0]
    return out


# ------------------------------------------------------------------------------------------------
# the detector
# ------------------------------------------------------------------------------------------------
class ImageBatchTransform(nn.Module):
    """torchvision's ``GeneralizedRCNNTransform`` for the detectors here: normalise, resize each image
    so its short side is ``min_size`` (long side <= ``max_size``), resize boxes / masks along, and pad
    the batch to a multiple of ``size_divisible`` (torchvision's 32 by default; a coarser bucket, e.g.
    128, keeps the set of conv shapes MIOpen sees small -- each new one costs a find)."""

    def __init__(self, min_size: int, max_size: int, size_divisible: int, channels_last: bool) -> None:
        super().__init__()
        self.size_divisible = max(32, int(size_divisible))
        self.min_size, self.max_size, self.channels_last = min_size, max_size, channels_last
        self.register_buffer("mean", torch.tensor(IMAGENET_MEAN).view(3, 1, 1), persistent=False)
        self.register_buffer("std", torch.tensor(IMAGENET_STD).view(3, 1, 1), persistent=False)

    def _transform(self, images: Sequence[torch.Tensor], targets: Optional[List[Dict[str, torch.Tensor]]]):
        dtype = next(p for p in self.parameters()).dtype
        resized, sizes, new_targets = [], [], []
        for i, img in enumerate(images):
            h, w = img.shape[-2:]
            scale = min(self.min_size / min(h, w), self.max_size / max(h, w))
            x = ((img.float() - self.mean.float()) / self.std.float())[None]
            x = F.interpolate(x, scale_factor=scale, mode="bilinear", recompute_scale_factor=True, align_corners=False)[0]
            resized.append(x)
            sizes.append((x.shape[-2], x.shape[-1]))
            if targets is not None:
                t = dict(targets[i])
                ry, rx = x.shape[-2] / h, x.shape[-1] / w
                t["boxes"] = t["boxes"].float() * torch.tensor([rx, ry, rx, ry], device=x.device)
                if "masks" in t:  # instance masks follow the image (nearest, as torchvision's transform)
                    mk = t["masks"]
                    t["masks"] = F.interpolate(mk[None].float(), size=x.shape[-2:], mode="nearest")[0].to(mk.dtype) \
                        if mk.numel() else mk.new_zeros((0,) + tuple(x.shape[-2:]))
                new_targets.append(t)
        d = self.size_divisible
        hm = (max(s[0] for s in sizes) + d - 1) // d * d
        wm = (max(s[1] for s in sizes) + d - 1) // d * d
        batch = resized[0].new_zeros(len(resized), 3, hm, wm)
        for i, x in enumerate(resized):
            batch[i, :, :x.shape[-2], :x.shape[-1]] = x
        batch = batch.to(dtype)
        if self.channels_last and batch.is_cuda:
            batch = batch.contiguous(memory_format=torch.channels_last)
        return batch, sizes, (new_targets if targets is not None else None)


class FasterRCNN(ImageBatchTransform):
    def __init__(self, num_classes: int = 91, min_size: int = 800, max_size: int = 1333, arch: str = "resnet50",
                 trainable_layers: int = 3, channels_last: bool = True, size_divisible: int = 32) -> None:
        super().__init__(min_size, max_size, size_divisible, channels_last)
        self.backbone = ResNetFPN(arch, trainable_layers)
        c = self.backbone.out_channels
        self.rpn = RPN(c, {"training": 2000, "testing": 1000}, {"training": 2000, "testing": 1000})
        self.roi_heads = self._make_roi_heads(c, num_classes)

    def _make_roi_heads(self, c: int, num_classes: int) -> RoIHeads:
        return RoIHeads(c, num_classes)

    def forward(self, images: Sequence[torch.Tensor], targets: Optional[List[Dict[str, torch.Tensor]]] = None):
        if self.training and targets is None:
            raise ValueError("targets are required in training mode")
        orig = [tuple(img.shape[-2:]) for img in images]
        batch, sizes, targets = self._transform(images, targets)
        feats = self.backbone(batch)
        image_hw = (batch.shape[-2], batch.shape[-1])
        proposals, rpn_losses = self.rpn(feats, image_hw, sizes, targets)
        dets, roi_losses = self.roi_heads(feats, proposals, image_hw, sizes, targets)
        if self.training:
            return {**roi_losses, **rpn_losses}
        for d, s, o in zip(dets, sizes, orig):
            ry, rx = o[0] / s[0], o[1] / s[1]
            d["boxes"] = d["boxes"] * torch.tensor([rx, ry, rx, ry], device=d["boxes"].device)
            if "masks" in d:  # per-box 28x28 probabilities pasted into the original image
                d["masks"] = paste_masks(d["masks"], d["boxes"], o)
        return dets
