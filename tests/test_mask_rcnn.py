"""Mask R-CNN pieces (models/mask_rcnn.py) on CPU: mask targets are the matched instance's mask
cropped to each RoI (RoIAlign over the stacked instance masks), the mask-head batch is bucketed,
and a tiny model trains (finite losses incl. loss_mask) and returns full-image masks in eval."""
import torch

from determined_1_amd.models.mask_rcnn import MaskRCNN, MaskRoIHeads


def test_mask_targets_crop_the_matched_instance():
    h, w = 64, 80
    m0 = torch.zeros(h, w, dtype=torch.uint8)
    m0[10:30, 20:60] = 1
    m1 = torch.zeros(h, w, dtype=torch.uint8)
    m1[40:60, 5:25] = 1
    targets = [{"masks": torch.stack([m0, m1])}]
    rois = torch.tensor([[0.0, 20, 10, 60, 30], [0.0, 5, 40, 25, 60], [0.0, 20, 10, 60, 30]])
    gid = torch.tensor([0, 1, 1])
    t = MaskRoIHeads._mask_targets(targets, rois, gid, (h, w), 28)
    assert t.shape == (3, 28, 28)
    # the box covers exactly its instance (the last sample row/column straddles the mask edge, as in
    # torchvision's aligned=False RoIAlign targets)
    assert float(t[0, :-1, :-1].min()) == 1.0 and float(t[1, :-1, :-1].min()) == 1.0
    assert float(t[2].max()) == 0.0  # instance 1 does not overlap RoI 0's box


def test_tiny_mask_rcnn_trains_and_predicts():
    torch.manual_seed(0)
    model = MaskRCNN(num_classes=3, min_size=64, max_size=96, arch="resnet26", mask_bucket=16)
    imgs = [torch.rand(3, 60, 72), torch.rand(3, 70, 50)]
    tg = []
    for img in imgs:
        h, w = img.shape[1:]
        mk = torch.zeros(2, h, w, dtype=torch.uint8)
        mk[0, 5:30, 5:40] = 1
        mk[1, 35:55, 10:30] = 1
        tg.append({"boxes": torch.tensor([[5.0, 5, 40, 30], [10.0, 35, 30, 55]]), "labels": torch.tensor([1, 2]),
                   "masks": mk})
    model.train()
    losses = model(imgs, tg)
    assert {"loss_mask", "loss_classifier", "loss_box_reg", "loss_objectness", "loss_rpn_box_reg"} <= set(losses)
    total = sum(losses.values())
    assert torch.isfinite(total)
    total.backward()
    assert model.roi_heads.mask_head.logits.weight.grad is not None
    model.eval()
    with torch.no_grad():
        out = model(imgs)
    for o, img in zip(out, imgs):
        assert o["masks"].shape[1:] == (1,) + tuple(img.shape[1:])
        assert o["masks"].shape[0] == o["boxes"].shape[0]


def test_synthetic_coco_instance_load():
    """instance_dist="coco": COCO train2017-like instance counts (mean 7.3, capped at 93) and small
    objects; masks, boxes and labels stay aligned after occlusion drops, every mask is non-empty
    and inside its box.  The default "uniform" load is unchanged (1..max_objects)."""
    from determined_1_amd.models.detection import SyntheticCocoInstances

    ds = SyntheticCocoInstances(150, min_size=200, max_size=260, instance_dist="coco")
    counts, small = [], 0
    for i in range(len(ds)):
        img, t = ds[i]
        n = t["labels"].shape[0]
        assert t["boxes"].shape == (n, 4) and t["masks"].shape[0] == n and n >= 1
        counts.append(n)
        areas = t["masks"].flatten(1).sum(1)
        assert bool((areas > 0).all())
        for b, m in zip(t["boxes"].tolist(), t["masks"]):
            ys, xs = torch.nonzero(m, as_tuple=True)
            assert xs.min() >= b[0] and xs.max() < b[2] and ys.min() >= b[1] and ys.max() < b[3]
        small += int(((t["boxes"][:, 2] - t["boxes"][:, 0]) * (t["boxes"][:, 3] - t["boxes"][:, 1]) < 32 * 32).sum())
    mean = sum(counts) / len(counts)
    assert 5.5 < mean < 8.5, mean  # geometric(1/7.3) less the fully occluded
    assert max(counts) > 15 and max(counts) <= SyntheticCocoInstances.COCO_MAX_INSTANCES
    assert small / sum(counts) > 0.2  # COCO: ~41 % small objects
    uni = SyntheticCocoInstances(50, min_size=200, max_size=260)
    assert all(1 <= uni[i][1]["labels"].shape[0] <= uni.max_objects for i in range(50))
