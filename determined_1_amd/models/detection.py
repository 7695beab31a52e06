"""Set-prediction detection machinery shared by the detection examples: box algebra, the Hungarian
matcher, DETR's set criterion, post-processing and a COCO-protocol bbox mAP evaluator.

Reference behaviour: ``examples/computer_vision/detr_coco_pytorch/model.py:33-233`` (SetCriterion:
labels / boxes / cardinality losses, aux-decoder losses with ``_<i>`` suffixes, ``num_boxes``
averaged over ranks and clamped at 1) and the upstream DETR matcher / box_ops / PostProcess it
imports; ``model_def.py:153-219`` (losses averaged over the validation set + COCO stats
``mAP, mAP_50, mAP_75, mAP_small, mAP_medium, mAP_large``).

MI355X-first differences:
  * the matcher builds the cost matrices of *all* decoder layers (final + aux) in one batched GPU
    computation and moves them to the host in ONE copy per step, instead of one synchronising
    transfer per layer per image; the Hungarian solve itself is scipy's ``linear_sum_assignment``
    (it is inherently sequential, so it stays on the CPU);
  * class / box losses of all decoder layers are computed as one stacked computation (one
    cross-entropy over ``[L*B, Q, C+1]``, one gather of matched boxes) -- a handful of kernels
    per step regardless of the number of aux layers;
  * the COCO evaluator is a self-contained numpy implementation of the pycocotools bbox protocol
    (pycocotools is not installed): greedy score-ordered matching per (image, category) at IoU
    thresholds .50:.05:.95, 101-point interpolated precision, area ranges small/medium/large,
    at most 100 detections per image.
"""
import math
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


# ------------------------------------------------------------------------------------------------
# boxes
# ------------------------------------------------------------------------------------------------
def box_cxcywh_to_xyxy(b: torch.Tensor) -> torch.Tensor:
    cx, cy, w, h = b.unbind(-1)
    return torch.stack([cx - 0.5 * w, cy - 0.5 * h, cx + 0.5 * w, cy + 0.5 * h], -1)


def box_xyxy_to_cxcywh(b: torch.Tensor) -> torch.Tensor:
    x0, y0, x1, y1 = b.unbind(-1)
    return torch.stack([(x0 + x1) / 2, (y0 + y1) / 2, x1 - x0, y1 - y0], -1)


def box_area(b: torch.Tensor) -> torch.Tensor:
    return (b[..., 2] - b[..., 0]) * (b[..., 3] - b[..., 1])


def box_iou(a: torch.Tensor, b: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Pairwise IoU of xyxy boxes ``a [..., N, 4]`` and ``b [..., M, 4]`` -> ``([..., N, M], union)``."""
    area_a, area_b = box_area(a), box_area(b)
    lt = torch.max(a[..., :, None, :2], b[..., None, :, :2])
    rb = torch.min(a[..., :, None, 2:], b[..., None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    union = area_a[..., :, None] + area_b[..., None, :] - inter
    return inter / union, union


def generalized_box_iou(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Pairwise GIoU (Rezatofighi et al. 2019) of xyxy boxes, batched over leading dims."""
    iou, union = box_iou(a, b)
    lt = torch.min(a[..., :, None, :2], b[..., None, :, :2])
    rb = torch.max(a[..., :, None, 2:], b[..., None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    hull = wh[..., 0] * wh[..., 1]
    return iou - (hull - union) / hull


def paired_giou(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """GIoU of matched pairs ``a[i]`` vs ``b[i]`` (the diagonal, without the N x N matrix)."""
    area_a, area_b = box_area(a), box_area(b)
    inter_wh = (torch.min(a[:, 2:], b[:, 2:]) - torch.max(a[:, :2], b[:, :2])).clamp(min=0)
    inter = inter_wh[:, 0] * inter_wh[:, 1]
    union = area_a + area_b - inter
    hull_wh = (torch.max(a[:, 2:], b[:, 2:]) - torch.min(a[:, :2], b[:, :2])).clamp(min=0)
    hull = hull_wh[:, 0] * hull_wh[:, 1]
    return inter / union - (hull - union) / hull


# ------------------------------------------------------------------------------------------------
# matching
# ------------------------------------------------------------------------------------------------
class HungarianMatcher(nn.Module):
    """Optimal one-to-one assignment of predictions to targets per image, minimising
    ``w_class * -p(class) + w_bbox * L1(cxcywh) + w_giou * -GIoU``."""

    def __init__(self, cost_class: float = 1.0, cost_bbox: float = 1.0, cost_giou: float = 1.0) -> None:
        super().__init__()
        assert cost_class or cost_bbox or cost_giou, "all matcher costs cannot be 0"
        self.cost_class, self.cost_bbox, self.cost_giou = cost_class, cost_bbox, cost_giou

    @torch.no_grad()
    def cost_matrices(self, logits: torch.Tensor, boxes: torch.Tensor, targets: Sequence[Dict[str, torch.Tensor]]
                      ) -> torch.Tensor:
        """``logits [L, B, Q, C+1]``, ``boxes [L, B, Q, 4]`` -> costs ``[L, B, Q, T_total]`` (all
        targets of the batch concatenated; each image later reads only its own column slice)."""
        tgt_ids = torch.cat([t["labels"] for t in targets])
        tgt_box = torch.cat([t["boxes"] for t in targets]).to(boxes.dtype)
        prob = logits.float().softmax(-1)
        c_class = -prob[..., tgt_ids]
        c_bbox = (boxes.float()[..., :, None, :] - tgt_box.float()).abs().sum(-1)
        c_giou = -generalized_box_iou(box_cxcywh_to_xyxy(boxes.float()), box_cxcywh_to_xyxy(tgt_box.float()))
        return self.cost_bbox * c_bbox + self.cost_class * c_class + self.cost_giou * c_giou

    @torch.no_grad()
    def match_all(self, logits: torch.Tensor, boxes: torch.Tensor, targets: Sequence[Dict[str, torch.Tensor]]
                  ) -> List[List[Tuple[torch.Tensor, torch.Tensor]]]:
        """Assignments for every decoder layer: ``out[l][b] = (pred_idx, tgt_idx)`` (int64, CPU)."""
        from scipy.optimize import linear_sum_assignment

        sizes = [int(t["boxes"].shape[0]) for t in targets]
        n_layers, n_img = logits.shape[0], logits.shape[1]
        if sum(sizes) == 0:
            empty = (torch.empty(0, dtype=torch.int64), torch.empty(0, dtype=torch.int64))
            return [[empty for _ in range(n_img)] for _ in range(n_layers)]
        c = self.cost_matrices(logits, boxes, targets).cpu().numpy()  # the one host sync of the step
        offs = np.concatenate([[0], np.cumsum(sizes)])
        out = []
        for layer in range(n_layers):
            per_img = []
            for b in range(n_img):
                sub = c[layer, b, :, offs[b]:offs[b + 1]]
                i, j = linear_sum_assignment(sub)
                per_img.append((torch.as_tensor(i, dtype=torch.int64), torch.as_tensor(j, dtype=torch.int64)))
            out.append(per_img)
        return out

    def forward(self, outputs: Dict[str, torch.Tensor], targets: Sequence[Dict[str, torch.Tensor]]
                ) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        return self.match_all(outputs["pred_logits"][None], outputs["pred_boxes"][None], targets)[0]


# ------------------------------------------------------------------------------------------------
# criterion
# ------------------------------------------------------------------------------------------------
class SetCriterion(nn.Module):
    """DETR losses: ``loss_ce`` (weighted CE, no-object weight ``eos_coef``), ``loss_bbox`` (L1),
    ``loss_giou``, logged ``class_error`` and ``cardinality_error``; aux decoder layers add the
    same keys suffixed ``_<i>`` (``class_error`` only for the final layer)."""

    def __init__(self, num_classes: int, matcher: HungarianMatcher, weight_dict: Dict[str, float], eos_coef: float,
                 losses: Sequence[str] = ("labels", "boxes", "cardinality")) -> None:
        super().__init__()
        self.num_classes = num_classes
        self.matcher = matcher
        self.weight_dict = weight_dict
        self.eos_coef = eos_coef
        self.losses = list(losses)
        w = torch.ones(num_classes + 1)
        w[-1] = eos_coef
        self.register_buffer("empty_weight", w)

    @staticmethod
    def _stack(outputs: Dict[str, Any]) -> Tuple[torch.Tensor, torch.Tensor]:
        """``[L, B, Q, *]`` with the final layer LAST (aux layers 0..L-2 first)."""
        aux = outputs.get("aux_outputs") or []
        logits = torch.stack([a["pred_logits"] for a in aux] + [outputs["pred_logits"]])
        boxes = torch.stack([a["pred_boxes"] for a in aux] + [outputs["pred_boxes"]])
        return logits, boxes

    def num_boxes(self, targets: Sequence[Dict[str, torch.Tensor]], device: torch.device, sync: bool) -> float:
        n = torch.tensor([float(sum(len(t["labels"]) for t in targets))], device=device)
        if sync and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(n)
            n /= dist.get_world_size()  # the reference averages (Horovod allreduce), then clamps
        return max(float(n.item()), 1.0)

    def forward(self, outputs: Dict[str, Any], targets: Sequence[Dict[str, torch.Tensor]], eval: bool = False
                ) -> Dict[str, torch.Tensor]:
        logits, boxes = self._stack(outputs)
        n_layers, n_img, n_q = logits.shape[:3]
        device = logits.device
        indices = self.matcher.match_all(logits.detach(), boxes.detach(), targets)
        num_boxes = self.num_boxes(targets, device, sync=not eval)

        # flat (layer, image, query) indices of every matched prediction, and its target row
        lid, bid, qid, tid = [], [], [], []
        offs = np.concatenate([[0], np.cumsum([len(t["labels"]) for t in targets])])
        for layer, per_img in enumerate(indices):
            for b, (src, tgt) in enumerate(per_img):
                lid.append(torch.full_like(src, layer))
                bid.append(torch.full_like(src, b))
                qid.append(src)
                tid.append(tgt + int(offs[b]))
        lid_t, bid_t, qid_t, tid_t = (torch.cat(v).to(device) for v in (lid, bid, qid, tid))
        tgt_labels = torch.cat([t["labels"] for t in targets]).to(device)
        tgt_boxes = torch.cat([t["boxes"] for t in targets]).to(device)

        per_layer: Dict[str, torch.Tensor] = {}
        if "labels" in self.losses:
            target_classes = torch.full((n_layers, n_img, n_q), self.num_classes, dtype=torch.int64, device=device)
            target_classes[lid_t, bid_t, qid_t] = tgt_labels[tid_t]
            ce = F.cross_entropy(logits.float().reshape(-1, logits.shape[-1]), target_classes.reshape(-1),
                                 self.empty_weight.to(device), reduction="none").view(n_layers, n_img * n_q)
            wsum = self.empty_weight.to(device)[target_classes].view(n_layers, -1).sum(1)
            per_layer["loss_ce"] = ce.sum(1) / wsum
        if "boxes" in self.losses:
            src = boxes.float()[lid_t, bid_t, qid_t]
            tgt = tgt_boxes.float()[tid_t]
            l1 = (src - tgt).abs().sum(1)
            giou = 1 - paired_giou(box_cxcywh_to_xyxy(src), box_cxcywh_to_xyxy(tgt))
            zeros = torch.zeros(n_layers, device=device)
            per_layer["loss_bbox"] = zeros.index_add(0, lid_t, l1) / num_boxes
            per_layer["loss_giou"] = zeros.index_add(0, lid_t, giou) / num_boxes
        if "cardinality" in self.losses:
            with torch.no_grad():
                tgt_len = torch.tensor([float(len(t["labels"])) for t in targets], device=device)
                card = (logits.argmax(-1) != logits.shape[-1] - 1).sum(-1).float()  # [L, B]
                per_layer["cardinality_error"] = (card - tgt_len).abs().mean(1)

        losses: Dict[str, torch.Tensor] = {}
        final = n_layers - 1
        for k, v in per_layer.items():
            losses[k] = v[final]
            for layer in range(final):
                losses[f"{k}_{layer}"] = v[layer]
        if "labels" in self.losses:
            with torch.no_grad():
                sel = lid_t == final
                if bool(sel.any()):
                    pred = logits[final][bid_t[sel], qid_t[sel]].argmax(-1)
                    acc = (pred == tgt_labels[tid_t[sel]]).float().mean() * 100
                else:
                    acc = torch.tensor(100.0, device=device)
                losses["class_error"] = 100 - acc
        return losses


# ------------------------------------------------------------------------------------------------
# post-processing and evaluation
# ------------------------------------------------------------------------------------------------
@torch.no_grad()
def postprocess(outputs: Dict[str, torch.Tensor], target_sizes: torch.Tensor) -> List[Dict[str, torch.Tensor]]:
    """Scores/labels/absolute xyxy boxes per image (``target_sizes [B, 2]`` as (h, w))."""
    prob = outputs["pred_logits"].float().softmax(-1)
    scores, labels = prob[..., :-1].max(-1)
    boxes = box_cxcywh_to_xyxy(outputs["pred_boxes"].float())
    h, w = target_sizes.float().unbind(1)
    boxes = boxes * torch.stack([w, h, w, h], 1)[:, None, :]
    return [{"scores": s, "labels": lab, "boxes": b} for s, lab, b in zip(scores, labels, boxes)]


AREA_RANGES = {"all": (0.0, 1e10), "small": (0.0, 32.0 ** 2), "medium": (32.0 ** 2, 96.0 ** 2),
               "large": (96.0 ** 2, 1e10)}
IOU_THRS = np.linspace(0.5, 0.95, 10)
REC_THRS = np.linspace(0.0, 1.0, 101)


def _np_iou(d: np.ndarray, g: np.ndarray) -> np.ndarray:
    if len(d) == 0 or len(g) == 0:
        return np.zeros((len(d), len(g)))
    lt = np.maximum(d[:, None, :2], g[None, :, :2])
    rb = np.minimum(d[:, None, 2:], g[None, :, 2:])
    wh = np.clip(rb - lt, 0, None)
    inter = wh[..., 0] * wh[..., 1]
    ad = (d[:, 2] - d[:, 0]) * (d[:, 3] - d[:, 1])
    ag = (g[:, 2] - g[:, 0]) * (g[:, 3] - g[:, 1])
    return inter / (ad[:, None] + ag[None, :] - inter)


class CocoBboxEvaluator:
    """Accumulates per-image detections and ground truth (absolute xyxy boxes), then
    ``summarize()`` returns the first six COCO bbox stats: AP@[.5:.95], AP50, AP75, AP small /
    medium / large (-1 where a category/area bucket has no ground truth, as pycocotools does)."""

    def __init__(self, max_dets: int = 100) -> None:
        self.max_dets = max_dets
        self.dets: Dict[int, Dict[str, np.ndarray]] = {}
        self.gts: Dict[int, Dict[str, np.ndarray]] = {}

    def add(self, image_id: int, pred: Dict[str, Any], gt_boxes_xyxy: Any, gt_labels: Any) -> None:
        def arr(x: Any) -> np.ndarray:
            return x.detach().float().cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x, dtype=np.float64)
        self.dets[int(image_id)] = {"boxes": arr(pred["boxes"]).reshape(-1, 4), "scores": arr(pred["scores"]).reshape(-1),
                                    "labels": arr(pred["labels"]).reshape(-1).astype(np.int64)}
        self.gts[int(image_id)] = {"boxes": arr(gt_boxes_xyxy).reshape(-1, 4),
                                   "labels": arr(gt_labels).reshape(-1).astype(np.int64)}

    def _evaluate(self, area: Tuple[float, float]) -> np.ndarray:
        """Precision ``[T, R, K]`` (IoU thresholds x recall points x categories), -1 = undefined."""
        cats = sorted({int(c) for g in self.gts.values() for c in g["labels"]} |
                      {int(c) for d in self.dets.values() for c in d["labels"]})
        precision = -np.ones((len(IOU_THRS), len(REC_THRS), len(cats)))
        for k, cat in enumerate(cats):
            scores_all, tp_all, fp_all, n_gt = [], [], [], 0
            for img in self.gts.keys() | self.dets.keys():
                g = self.gts.get(img, {"boxes": np.zeros((0, 4)), "labels": np.zeros(0, np.int64)})
                d = self.dets.get(img, {"boxes": np.zeros((0, 4)), "scores": np.zeros(0), "labels": np.zeros(0, np.int64)})
                gb = g["boxes"][g["labels"] == cat]
                dm = d["labels"] == cat
                db, ds = d["boxes"][dm], d["scores"][dm]
                order = np.argsort(-ds, kind="mergesort")[:self.max_dets]
                db, ds = db[order], ds[order]
                ga = (gb[:, 2] - gb[:, 0]) * (gb[:, 3] - gb[:, 1])
                g_ignore = (ga < area[0]) | (ga > area[1])
                g_order = np.argsort(g_ignore, kind="mergesort")  # non-ignored ground truth first
                gb, g_ignore = gb[g_order], g_ignore[g_order]
                n_gt += int((~g_ignore).sum())
                ious = _np_iou(db, gb)
                da = (db[:, 2] - db[:, 0]) * (db[:, 3] - db[:, 1])
                tp = np.zeros((len(IOU_THRS), len(db)))
                d_ignore = np.zeros((len(IOU_THRS), len(db)), dtype=bool)
                for t, thr in enumerate(IOU_THRS):
                    taken = np.zeros(len(gb), dtype=bool)
                    for di in range(len(db)):
                        best, m = min(thr, 1 - 1e-10), -1
                        for gi in range(len(gb)):
                            if taken[gi]:
                                continue
                            if m > -1 and not g_ignore[m] and g_ignore[gi]:
                                break  # a matched real gt beats any ignored one
                            if ious[di, gi] < best:
                                continue
                            best, m = ious[di, gi], gi
                        if m == -1:
                            continue
                        taken[m] = True
                        d_ignore[t, di] = g_ignore[m]
                        tp[t, di] = 1
                    out_of_range = (da < area[0]) | (da > area[1])
                    d_ignore[t] |= (tp[t] == 0) & out_of_range
                scores_all.append(ds)
                tp_all.append(np.where(d_ignore, 0, tp))
                fp_all.append(np.where(d_ignore, 0, 1 - tp))
            if n_gt == 0:
                continue
            s = np.concatenate(scores_all) if scores_all else np.zeros(0)
            order = np.argsort(-s, kind="mergesort")
            tps = np.concatenate(tp_all, 1)[:, order] if tp_all else np.zeros((len(IOU_THRS), 0))
            fps = np.concatenate(fp_all, 1)[:, order] if fp_all else np.zeros((len(IOU_THRS), 0))
            for t in range(len(IOU_THRS)):
                tp_c, fp_c = np.cumsum(tps[t]), np.cumsum(fps[t])
                rc = tp_c / n_gt
                pr = tp_c / np.maximum(tp_c + fp_c, np.spacing(1))
                for i in range(len(pr) - 1, 0, -1):  # precision envelope
                    pr[i - 1] = max(pr[i - 1], pr[i])
                q = np.zeros(len(REC_THRS))
                idx = np.searchsorted(rc, REC_THRS, side="left")
                for ri, pi in enumerate(idx):
                    if pi < len(pr):
                        q[ri] = pr[pi]
                precision[t, :, k] = q
        return precision

    @staticmethod
    def _mean(p: np.ndarray) -> float:
        v = p[p > -1]
        return float(v.mean()) if v.size else -1.0

    def summarize(self) -> List[float]:
        p_all = self._evaluate(AREA_RANGES["all"])
        stats = [self._mean(p_all), self._mean(p_all[0]), self._mean(p_all[5])]
        for name in ("small", "medium", "large"):
            stats.append(self._mean(self._evaluate(AREA_RANGES[name])))
        return stats


# ------------------------------------------------------------------------------------------------
# synthetic COCO-shaped data
# ------------------------------------------------------------------------------------------------
class SyntheticDetection(torch.utils.data.Dataset):
    """COCO-shaped detection samples without a download: images of varying size (so batches need
    padding masks, as real COCO batches do) holding 1..``max_objects`` axis-aligned objects, each a
    rectangle filled with its class's colour over a noisy background.  Targets follow DETR's
    convention: ``boxes`` normalised cxcywh, ``labels`` in ``[1, num_classes)``, ``orig_size`` /
    ``size`` as (h, w), ``image_id``.  Deterministic per index."""

    def __init__(self, length: int, num_classes: int = 91, min_size: int = 96, max_size: int = 128,
                 max_objects: int = 6, seed: int = 0) -> None:
        self.length, self.num_classes = length, num_classes
        self.min_size, self.max_size, self.max_objects, self.seed = min_size, max_size, max_objects, seed
        g = torch.Generator().manual_seed(1234)
        self.colors = torch.rand(num_classes, 3, generator=g) * 2 - 1  # normalised-space class colours

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, idx: int) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + idx)
        h = int(torch.randint(self.min_size, self.max_size + 1, (1,), generator=g))
        w = int(torch.randint(self.min_size, self.max_size + 1, (1,), generator=g))
        img = torch.randn(3, h, w, generator=g) * 0.3
        n = int(torch.randint(1, self.max_objects + 1, (1,), generator=g))
        boxes, labels = [], []
        for _ in range(n):
            bw = int(torch.randint(max(4, w // 8), max(5, w // 2), (1,), generator=g))
            bh = int(torch.randint(max(4, h // 8), max(5, h // 2), (1,), generator=g))
            x0 = int(torch.randint(0, w - bw + 1, (1,), generator=g))
            y0 = int(torch.randint(0, h - bh + 1, (1,), generator=g))
            c = int(torch.randint(1, self.num_classes, (1,), generator=g))
            img[:, y0:y0 + bh, x0:x0 + bw] = self.colors[c].view(3, 1, 1)
            boxes.append([x0, y0, x0 + bw, y0 + bh])
            labels.append(c)
        xyxy = torch.tensor(boxes, dtype=torch.float32)
        scale = torch.tensor([w, h, w, h], dtype=torch.float32)
        target = {"boxes": box_xyxy_to_cxcywh(xyxy / scale), "labels": torch.tensor(labels, dtype=torch.int64),
                  "image_id": torch.tensor([idx]), "orig_size": torch.tensor([h, w]), "size": torch.tensor([h, w])}
        return img, target


class SyntheticCocoInstances(torch.utils.data.Dataset):
    """Synthetic COCO-shaped instance-segmentation data (the COCO download is unavailable offline):
    images of ``min_size``-``max_size`` px per side (landscape and portrait), filled ellipses or
    rectangles of a per-class colour over a noisy background, with absolute xyxy ``boxes``,
    ``labels`` and uint8 instance ``masks``.  Deterministic per index; images are float RGB in
    [0, 1] (the detectors normalise them themselves).

    ``instance_dist``: "uniform" = 1-``max_objects`` large instances (w/10-w/2 per side);
    "coco" = COCO train2017-like load: a geometric instance count with COCO's mean of 7.3 per
    image, capped at 93 (COCO's maximum), and log-uniform object areas from 8x8 px to half the
    image (COCO is ~41 % small objects), aspect ratios 1:2-2:1.  Later instances occlude earlier
    ones; fully occluded instances are dropped."""

    COCO_MEAN_INSTANCES = 7.3
    COCO_MAX_INSTANCES = 93

    def __init__(self, length: int, num_classes: int = 81, min_size: int = 480, max_size: int = 640,
                 max_objects: int = 6, seed: int = 0, instance_dist: str = "uniform") -> None:
        if instance_dist not in ("uniform", "coco"):
            raise ValueError(f"instance_dist must be 'uniform' or 'coco', got {instance_dist!r}")
        self.length, self.num_classes, self.min_size, self.max_size = length, num_classes, min_size, max_size
        self.max_objects, self.seed, self.instance_dist = max_objects, seed, instance_dist
        self.colors = torch.rand(num_classes, 3, generator=torch.Generator().manual_seed(4321))

    def _coco_boxes(self, g: torch.Generator, h: int, w: int) -> List[Tuple[int, int, int, int]]:
        p = 1.0 / self.COCO_MEAN_INSTANCES
        u = float(torch.rand(1, generator=g)) or 1e-12
        n = min(self.COCO_MAX_INSTANCES, 1 + int(math.log(u) / math.log(1.0 - p)))
        lo, hi = math.log(64.0 / (h * w)), math.log(0.25)  # area fraction: 8x8 px .. (1/2)^2
        out = []
        for _ in range(n):
            a, r = torch.rand(2, generator=g).tolist()
            area = math.exp(lo + a * (hi - lo)) * h * w
            ar = math.exp((r - 0.5) * 2 * math.log(2.0))
            bw = int(min(w, max(4, round(math.sqrt(area * ar)))))
            bh = int(min(h, max(4, round(math.sqrt(area / ar)))))
            x0 = int(torch.randint(0, w - bw + 1, (1,), generator=g))
            y0 = int(torch.randint(0, h - bh + 1, (1,), generator=g))
            c = int(torch.randint(1, self.num_classes, (1,), generator=g))
            out.append((x0, y0, bw, bh, c, float(torch.rand(1, generator=g)) < 0.5))
        return out

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, idx: int) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + idx)
        h = int(torch.randint(self.min_size, self.max_size + 1, (1,), generator=g))
        w = int(torch.randint(self.min_size, self.max_size + 1, (1,), generator=g))
        img = torch.rand(3, h, w, generator=g) * 0.2 + 0.4
        if self.instance_dist == "coco":
            geo = self._coco_boxes(g, h, w)
        else:
            geo = []
            for _ in range(int(torch.randint(1, self.max_objects + 1, (1,), generator=g))):
                bw = int(torch.randint(max(8, w // 10), max(9, w // 2), (1,), generator=g))
                bh = int(torch.randint(max(8, h // 10), max(9, h // 2), (1,), generator=g))
                x0 = int(torch.randint(0, w - bw + 1, (1,), generator=g))
                y0 = int(torch.randint(0, h - bh + 1, (1,), generator=g))
                c = int(torch.randint(1, self.num_classes, (1,), generator=g))
                geo.append((x0, y0, bw, bh, c, float(torch.rand(1, generator=g)) < 0.5))
        # owner map: later instances occlude earlier ones (O(n * box area), not O(n^2 * image))
        owner = torch.full((h, w), -1, dtype=torch.int16)
        boxes, labels = [], []
        for i, (x0, y0, bw, bh, c, ellipse) in enumerate(geo):
            if ellipse:  # inscribed in the box
                yy = torch.arange(bh).view(bh, 1).float() + 0.5 - bh / 2
                xx = torch.arange(bw).view(1, bw).float() + 0.5 - bw / 2
                m = ((yy / (bh / 2)) ** 2 + (xx / (bw / 2)) ** 2) <= 1.0
            else:
                m = torch.ones(bh, bw, dtype=torch.bool)
            sub = img[:, y0:y0 + bh, x0:x0 + bw]
            sub[:, m] = self.colors[c].view(3, 1)
            owner[y0:y0 + bh, x0:x0 + bw][m] = i
            boxes.append([float(x0), float(y0), float(x0 + bw), float(y0 + bh)])
            labels.append(c)
        ids = torch.arange(len(geo), dtype=torch.int16).view(-1, 1, 1)
        mk = (owner.unsqueeze(0) == ids).to(torch.uint8)
        keep = mk.flatten(1).sum(1) > 0  # fully occluded instances are dropped
        if not bool(keep.all()):
            mk = mk[keep]
            boxes = [b for b, k in zip(boxes, keep.tolist()) if k]
            labels = [c for c, k in zip(labels, keep.tolist()) if k]
        target = {"boxes": torch.tensor(boxes), "labels": torch.tensor(labels, dtype=torch.int64), "masks": mk,
                  "image_id": torch.tensor([idx])}
        return img, target


def pad_collate(batch: Sequence[Tuple[torch.Tensor, Dict[str, torch.Tensor]]],
                multiple: int = 32) -> Tuple[Dict[str, torch.Tensor], List]:
    """Pad a list of ``[3, h, w]`` images to the batch max (rounded up to ``multiple``, at least the
    backbone stride 32) and return ``({"tensors": [B,3,H,W], "mask": [B,H,W] True on padding},
    targets)`` -- the reference's ``unwrap_collate_fn`` layout.  A coarser ``multiple`` (e.g. 128)
    buckets the padded shapes: the masked padding changes nothing the model reads, but far fewer
    distinct conv shapes reach MIOpen (each new one costs a find / kernel build)."""
    multiple = max(32, int(multiple))
    imgs, targets = zip(*batch)
    hm = max(i.shape[1] for i in imgs)
    wm = max(i.shape[2] for i in imgs)
    hm, wm = (hm + multiple - 1) // multiple * multiple, (wm + multiple - 1) // multiple * multiple
    t = imgs[0].new_zeros(len(imgs), 3, hm, wm)
    mask = torch.ones(len(imgs), hm, wm, dtype=torch.bool)
    for k, im in enumerate(imgs):
        t[k, :, :im.shape[1], :im.shape[2]] = im
        mask[k, :im.shape[1], :im.shape[2]] = False
    return {"tensors": t, "mask": mask}, list(targets)


def list_collate(batch):
    """``[(image, target), ...]`` -> ``(images, targets)`` tuples (torchvision detection convention)."""
    return tuple(zip(*batch))
