"""Synthetic stand-in for PennFudanPed (reference ``fasterrcnn_coco_pytorch/data.py``: images of a
few hundred pixels, boxes around upright pedestrians, label 1).  Deterministic per index; images are
float RGB in [0, 1] (the detector normalises them itself, as torchvision's transform does)."""
from typing import Dict, List, Tuple

import torch


class SyntheticPedestrians(torch.utils.data.Dataset):
    def __init__(self, length: int, min_size: int = 300, max_size: int = 500, max_people: int = 4, seed: int = 0) -> None:
        self.length, self.min_size, self.max_size, self.max_people, self.seed = length, min_size, max_size, max_people, seed

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, idx: int) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
        g = torch.Generator().manual_seed(self.seed * 7919 + idx)
        h = int(torch.randint(self.min_size, self.max_size + 1, (1,), generator=g))
        w = int(torch.randint(self.min_size, self.max_size + 1, (1,), generator=g))
        img = (torch.rand(3, h, w, generator=g) * 0.3 + 0.35)
        n = int(torch.randint(1, self.max_people + 1, (1,), generator=g))
        boxes: List[List[float]] = []
        for _ in range(n):
            bh = int(torch.randint(h // 3, max(h // 3 + 1, int(h * 0.9)), (1,), generator=g))
            bw = max(4, int(bh * float(torch.empty(1).uniform_(0.3, 0.5, generator=g))))
            bw = min(bw, w - 1)
            x0 = int(torch.randint(0, w - bw, (1,), generator=g))
            y0 = int(torch.randint(0, h - bh, (1,), generator=g))
            color = torch.rand(3, 1, 1, generator=g)
            img[:, y0:y0 + bh, x0:x0 + bw] = color
            img[:, y0:y0 + bh // 6, x0 + bw // 4:x0 + 3 * bw // 4] = 1.0 - color  # a "head"
            boxes.append([float(x0), float(y0), float(x0 + bw), float(y0 + bh)])
        b = torch.tensor(boxes)
        target = {"boxes": b, "labels": torch.ones(n, dtype=torch.int64), "image_id": torch.tensor([idx]),
                  "area": (b[:, 3] - b[:, 1]) * (b[:, 2] - b[:, 0]), "iscrowd": torch.zeros(n, dtype=torch.int64)}
        return img, target


def collate_fn(batch):
    return tuple(zip(*batch))
