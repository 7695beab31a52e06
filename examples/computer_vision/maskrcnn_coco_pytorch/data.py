"""Synthetic COCO-shaped instance-segmentation data (the COCO download is unavailable offline):
images of 480-640 px per side (landscape and portrait), 1-6 instances each -- filled ellipses or
rectangles of a per-class colour over a noisy background -- with xyxy boxes, labels and uint8
instance masks.  Deterministic per index."""
from typing import Dict, Tuple

import torch


class SyntheticCocoInstances(torch.utils.data.Dataset):
    def __init__(self, length: int, num_classes: int = 81, min_size: int = 480, max_size: int = 640,
                 max_objects: int = 6, seed: int = 0) -> None:
        self.length, self.num_classes, self.min_size, self.max_size = length, num_classes, min_size, max_size
        self.max_objects, self.seed = max_objects, seed
        self.colors = torch.rand(num_classes, 3, generator=torch.Generator().manual_seed(4321))

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, idx: int) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + idx)
        h = int(torch.randint(self.min_size, self.max_size + 1, (1,), generator=g))
        w = int(torch.randint(self.min_size, self.max_size + 1, (1,), generator=g))
        img = torch.rand(3, h, w, generator=g) * 0.2 + 0.4
        n = int(torch.randint(1, self.max_objects + 1, (1,), generator=g))
        yy = torch.arange(h).view(h, 1).float()
        xx = torch.arange(w).view(1, w).float()
        boxes, labels, masks = [], [], []
        for _ in range(n):
            bw = int(torch.randint(max(8, w // 10), max(9, w // 2), (1,), generator=g))
            bh = int(torch.randint(max(8, h // 10), max(9, h // 2), (1,), generator=g))
            x0 = int(torch.randint(0, w - bw + 1, (1,), generator=g))
            y0 = int(torch.randint(0, h - bh + 1, (1,), generator=g))
            c = int(torch.randint(1, self.num_classes, (1,), generator=g))
            if float(torch.rand(1, generator=g)) < 0.5:  # ellipse inscribed in the box
                cy, cx, ry, rx = y0 + bh / 2, x0 + bw / 2, bh / 2, bw / 2
                m = (((yy + 0.5 - cy) / ry) ** 2 + ((xx + 0.5 - cx) / rx) ** 2) <= 1.0
            else:
                m = torch.zeros(h, w, dtype=torch.bool)
                m[y0:y0 + bh, x0:x0 + bw] = True
            img[:, m] = self.colors[c].view(3, 1)
            for prev in masks:  # later instances occlude earlier ones
                prev &= ~m
            masks.append(m)
            boxes.append([float(x0), float(y0), float(x0 + bw), float(y0 + bh)])
            labels.append(c)
        mk = torch.stack(masks).to(torch.uint8)
        target = {"boxes": torch.tensor(boxes), "labels": torch.tensor(labels, dtype=torch.int64), "masks": mk,
                  "image_id": torch.tensor([idx])}
        return img, target


def collate_fn(batch):
    return tuple(zip(*batch))
