"""det_detect.hip kernels vs the fp32 PyTorch references (ops/detect.py): multi-level RoIAlign
forward / backward (fp32 and bf16 maps) and device NMS (several 64-box blocks, ties, batched)."""
import pytest
import torch

from determined_1_amd.ops import detect

pytestmark = pytest.mark.gpu


def _feats(dtype, g):
    shapes = [(2, 32, 40, 48), (2, 32, 20, 24), (2, 32, 10, 12), (2, 32, 5, 6)]
    return [torch.randn(s, generator=g).to(dtype).to(memory_format=torch.channels_last) for s in shapes]


def _rois(g, k=300):
    xy = torch.rand(k, 2, generator=g) * torch.tensor([180.0, 150.0]) - 10
    wh = torch.rand(k, 2, generator=g) ** 2 * 900 + 0.5  # spread over all four pyramid levels
    b = torch.randint(0, 2, (k, 1), generator=g).float()
    return torch.cat([b, xy, xy + wh], 1)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_roi_align_fwd_bwd_matches_reference(gpu, dtype):
    g = torch.Generator().manual_seed(0)
    feats = _feats(dtype, g)
    rois = _rois(g)
    levels = detect.map_levels(rois[:, 1:], 2, 5)
    scales = [0.25, 0.125, 0.0625, 0.03125]
    ref_in = [f.detach().float().clone().requires_grad_(True) for f in feats]
    ref = detect.roi_align_multilevel(ref_in, rois, levels, scales, 7, 2)
    dy = torch.randn(ref.shape, generator=g)
    ref.backward(dy)

    gin = [f.detach().cuda().requires_grad_(True) for f in feats]
    out = detect.roi_align_multilevel(gin, rois.cuda(), levels.cuda(), scales, 7, 2)
    assert detect.COUNTS["roi_align_native"] > 0
    # sample positions are computed in a different (equally valid) fp32 order than the reference,
    # so fp32 agreement is ~1e-6 relative, not bitwise
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    err = (out.float().cpu() - ref.detach()).abs().max().item()
    assert err <= tol * (1 + ref.abs().max().item()), err
    out.backward(dy.to(dtype).cuda())
    for a, b in zip(gin, ref_in):
        gtol = 1e-4 if dtype == torch.float32 else 5e-2
        bg = b.grad if b.grad is not None else torch.zeros_like(b)  # a level no RoI maps to
        assert a.grad is not None
        gerr = (a.grad.float().cpu() - bg).abs().max().item()
        assert gerr <= gtol * (1 + bg.abs().max().item()), gerr


@pytest.mark.parametrize("n", [1, 63, 64, 65, 700, 5000])
def test_nms_matches_reference(gpu, n):
    g = torch.Generator().manual_seed(n)
    xy = torch.rand(n, 2, generator=g) * 400
    wh = torch.rand(n, 2, generator=g) * 60 + 1
    boxes = torch.cat([xy, xy + wh], 1)
    scores = torch.rand(n, generator=g)
    scores[: n // 3] = scores[n // 3: 2 * (n // 3)]  # ties: stable order decides
    want = detect._nms_ref(boxes, scores, 0.5)
    got = detect.nms(boxes.cuda(), scores.cuda(), 0.5).cpu()
    assert got.tolist() == want.tolist()


def test_batched_nms_on_gpu(gpu):
    g = torch.Generator().manual_seed(3)
    xy = torch.rand(400, 2, generator=g) * 100
    boxes = torch.cat([xy, xy + 30], 1)
    scores = torch.rand(400, generator=g)
    cls = torch.randint(0, 5, (400,), generator=g)
    want = detect.batched_nms(boxes, scores, cls, 0.4)
    got = detect.batched_nms(boxes.cuda(), scores.cuda(), cls.cuda(), 0.4).cpu()
    assert got.tolist() == want.tolist()
