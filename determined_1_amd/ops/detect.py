"""Detection ops on the hand-written kernels of ``csrc/det_detect.hip``: multi-level RoIAlign over
channels_last FPN maps (one launch for all levels, fwd + bwd) and device-side NMS.

Semantics follow torchvision's ``roi_align(aligned=False)`` / ``MultiScaleRoIAlign`` and
``nms`` / ``batched_nms``, which the reference's Faster R-CNN example uses
(``examples/computer_vision/fasterrcnn_coco_pytorch/model_def.py:18,48,112``); torchvision is not
in this image.  The pooled layout is ``[K, PH, PW, C]`` (see the kernel file header).

CPU tensors use the pure-PyTorch reference implementations below (also the numerics references
of the GPU tests); on a GPU tensor the HIP library is required (``_lib`` raises if it is missing).
"""
import ctypes
from typing import List, Sequence

import torch

from determined_1_amd.ops import _lib

_DT = {torch.float32: 0, torch.bfloat16: 1}
COUNTS = {"roi_align_native": 0, "nms_native": 0}


def _stream(t: torch.Tensor) -> int:
    return torch._C._cuda_getCurrentRawStream(t.device.index)


# ------------------------------------------------------------------------------------------------
# RoIAlign
# ------------------------------------------------------------------------------------------------
def _roi_align_ref_level(feat: torch.Tensor, rois: torch.Tensor, scale: float, ph: int, pw: int, s: int) -> torch.Tensor:
    """Reference RoIAlign (aligned=False, fixed sampling ``s``) of NHWC ``feat`` -> [K, ph, pw, C]."""
    n, h, w, c = feat.shape
    k = rois.shape[0]
    if k == 0:
        return feat.new_zeros(0, ph, pw, c)
    r = rois.float()
    x1, y1 = r[:, 1] * scale, r[:, 2] * scale
    rw = (r[:, 3] * scale - x1).clamp(min=1.0)
    rh = (r[:, 4] * scale - y1).clamp(min=1.0)
    ys = y1[:, None] + (torch.arange(ph * s, dtype=torch.float32, device=feat.device) + 0.5) * (rh / ph / s)[:, None]
    xs = x1[:, None] + (torch.arange(pw * s, dtype=torch.float32, device=feat.device) + 0.5) * (rw / pw / s)[:, None]

    def axis(v: torch.Tensor, size: int):
        valid = (v >= -1.0) & (v <= size)
        v = v.clamp(min=0.0)
        lo = v.floor().long()
        at_edge = lo >= size - 1
        lo = torch.where(at_edge, torch.full_like(lo, size - 1), lo)
        hi = torch.where(at_edge, lo, lo + 1)
        v = torch.where(at_edge, lo.float(), v)
        frac = v - lo.float()
        return lo, hi, frac, valid

    yl, yh, ly, vy = axis(ys, h)
    xl, xh, lx, vx = axis(xs, w)
    b = r[:, 0].long()[:, None, None]
    f = feat.float()

    def g(yy, xx):
        return f[b, yy[:, :, None], xx[:, None, :]]  # [K, PH*s, PW*s, C]

    wy1, wy0 = ly[:, :, None, None], (1 - ly)[:, :, None, None]
    wx1, wx0 = lx[:, None, :, None], (1 - lx)[:, None, :, None]
    val = wy0 * wx0 * g(yl, xl) + wy0 * wx1 * g(yl, xh) + wy1 * wx0 * g(yh, xl) + wy1 * wx1 * g(yh, xh)
    val = val * (vy[:, :, None, None] & vx[:, None, :, None]).float()
    return val.view(k, ph, s, pw, s, c).mean(dim=(2, 4)).to(feat.dtype)


class _RoIAlignMulti(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rois, levels, scales, out_hw, sampling, *feats):
        ph, pw = out_hw
        k = rois.shape[0]
        c = feats[0].shape[-1]
        dtype = feats[0].dtype
        out = torch.empty(k, ph, pw, c, dtype=dtype, device=rois.device)
        rois_c = rois.float().contiguous()
        lv = levels.to(torch.int32).contiguous()
        n_l = len(feats)
        fp = _arr(ctypes.c_void_p, [f.data_ptr() for f in feats])
        hs = _arr(ctypes.c_int, [f.shape[1] for f in feats])
        ws = _arr(ctypes.c_int, [f.shape[2] for f in feats])
        sc = _arr(ctypes.c_float, list(scales))
        _lib.check(_lib.get_lib().det_roi_align_fwd(_stream(rois), _DT[dtype], rois_c.data_ptr(), lv.data_ptr(), k, n_l,
                                                    fp, hs, ws, sc, c, ph, pw, sampling, out.data_ptr()),
                   "det_roi_align_fwd")
        ctx.save_for_backward(rois_c, lv)
        ctx.meta = ([tuple(f.shape) for f in feats], list(scales), (ph, pw), sampling, dtype)
        COUNTS["roi_align_native"] += 1
        return out

    @staticmethod
    def backward(ctx, dy):
        rois_c, lv = ctx.saved_tensors
        shapes, scales, (ph, pw), sampling, dtype = ctx.meta
        dy = dy.contiguous().to(dtype)
        grads = [torch.zeros(s, dtype=torch.float32, device=dy.device) for s in shapes]
        gp = _arr(ctypes.c_void_p, [g.data_ptr() for g in grads])
        hs = _arr(ctypes.c_int, [s[1] for s in shapes])
        ws = _arr(ctypes.c_int, [s[2] for s in shapes])
        sc = _arr(ctypes.c_float, scales)
        _lib.check(_lib.get_lib().det_roi_align_bwd(_stream(dy), _DT[dtype], rois_c.data_ptr(), lv.data_ptr(),
                                                    rois_c.shape[0], len(shapes), gp, hs, ws, sc, shapes[0][-1], ph, pw,
                                                    sampling, dy.data_ptr()), "det_roi_align_bwd")
        return (None, None, None, None, None) + tuple(g.to(dtype) for g in grads)


def _arr(ctype, vals):
    return (ctype * len(vals))(*vals)


def roi_align_multilevel(feats: Sequence[torch.Tensor], rois: torch.Tensor, levels: torch.Tensor,
                         scales: Sequence[float], output_size: int = 7, sampling_ratio: int = 2) -> torch.Tensor:
    """Pool ``rois [K, 5]`` (batch index, x1, y1, x2, y2 in image coordinates) from the level each
    is assigned to (``levels [K]``, indices into ``feats``).  ``feats`` are ``[N, C, H, W]``
    tensors in channels_last memory format (or NHWC-contiguous).  Returns ``[K, PH, PW, C]``."""
    nhwc = [f.permute(0, 2, 3, 1) for f in feats]  # a view for channels_last tensors
    if rois.device.type == "cuda":
        if sampling_ratio <= 0:
            raise ValueError("sampling_ratio must be > 0")
        nhwc = [f.contiguous() for f in nhwc]
        if nhwc[0].dtype not in _DT or len({f.dtype for f in nhwc}) != 1:
            raise TypeError(f"roi_align: unsupported feature dtype {nhwc[0].dtype}")
        return _RoIAlignMulti.apply(rois, levels, tuple(float(s) for s in scales), (output_size, output_size),
                                    int(sampling_ratio), *nhwc)
    c = nhwc[0].shape[-1]
    out = nhwc[0].new_zeros(rois.shape[0], output_size, output_size, c)
    for lvl, (f, s) in enumerate(zip(nhwc, scales)):
        idx = torch.nonzero(levels == lvl).flatten()
        if idx.numel():
            out = out.index_put((idx,), _roi_align_ref_level(f, rois[idx], float(s), output_size, output_size,
                                                             sampling_ratio))
    return out


def map_levels(boxes: torch.Tensor, k_min: int, k_max: int, canonical_scale: float = 224.0,
               canonical_level: int = 4) -> torch.Tensor:
    """FPN level of each box (Lin et al. 2017, eq. 1; torchvision LevelMapper) as an index from 0."""
    area = ((boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1])).clamp(min=0)
    lvl = torch.floor(canonical_level + torch.log2(area.sqrt() / canonical_scale + 1e-6))
    return (lvl.clamp(k_min, k_max) - k_min).to(torch.int64)


# ------------------------------------------------------------------------------------------------
# NMS
# ------------------------------------------------------------------------------------------------
def pairwise_iou(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    area_a = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
    area_b = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    lt = torch.max(a[:, None, :2], b[None, :, :2])
    rb = torch.min(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    union = area_a[:, None] + area_b[None, :] - inter
    return torch.where(union > 0, inter / union, torch.zeros_like(inter))


def _nms_ref(boxes: torch.Tensor, scores: torch.Tensor, thr: float) -> torch.Tensor:
    order = torch.sort(scores, descending=True, stable=True).indices
    b = boxes[order].float()
    iou = pairwise_iou(b, b)
    n = b.shape[0]
    removed = torch.zeros(n, dtype=torch.bool)
    keep = []
    for i in range(n):
        if removed[i]:
            continue
        keep.append(i)
        removed |= iou[i] > thr
        removed[i] = True
    return order[torch.tensor(keep, dtype=torch.int64)] if keep else order[:0]


def nms(boxes: torch.Tensor, scores: torch.Tensor, iou_threshold: float) -> torch.Tensor:
    """Indices of the boxes kept by greedy NMS, in decreasing score order (torchvision.ops.nms)."""
    if boxes.numel() == 0:
        return torch.empty(0, dtype=torch.int64, device=boxes.device)
    if boxes.device.type != "cuda":
        return _nms_ref(boxes, scores, iou_threshold)
    n = boxes.shape[0]
    lib = _lib.get_lib()
    if n > lib.det_nms_max_boxes():
        raise ValueError(f"nms: {n} boxes exceeds the kernel limit {lib.det_nms_max_boxes()}")
    order = torch.sort(scores, descending=True, stable=True).indices
    b = boxes[order].float().contiguous()
    cb = lib.det_nms_mask_words(n)
    mask = torch.empty(n * cb, dtype=torch.int64, device=boxes.device)
    keep = torch.empty(n, dtype=torch.uint8, device=boxes.device)
    _lib.check(lib.det_nms(_stream(b), b.data_ptr(), n, float(iou_threshold), mask.data_ptr(), keep.data_ptr()),
               "det_nms")
    COUNTS["nms_native"] += 1
    return order[keep.bool()]


def batched_nms(boxes: torch.Tensor, scores: torch.Tensor, idxs: torch.Tensor, iou_threshold: float) -> torch.Tensor:
    """NMS independently per category ``idxs`` in one pass: boxes of different categories are
    shifted apart so they never overlap (torchvision's coordinate trick)."""
    if boxes.numel() == 0:
        return torch.empty(0, dtype=torch.int64, device=boxes.device)
    offsets = idxs.to(boxes.dtype) * (boxes.max() + 1)
    return nms(boxes + offsets[:, None], scores, iou_threshold)


def remove_small_boxes(boxes: torch.Tensor, min_size: float) -> torch.Tensor:
    ws, hs = boxes[:, 2] - boxes[:, 0], boxes[:, 3] - boxes[:, 1]
    return torch.nonzero((ws >= min_size) & (hs >= min_size)).flatten()


def clip_boxes_to_image(boxes: torch.Tensor, size: List[int]) -> torch.Tensor:
    h, w = size
    x = boxes[..., 0::2].clamp(min=0, max=w)
    y = boxes[..., 1::2].clamp(min=0, max=h)
    return torch.stack((x, y), dim=-1).reshape(boxes.shape)
