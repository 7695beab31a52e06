"""Prototypical networks (Snell et al. 2017) few-shot classification PyTorchTrial.

Mirrors the reference's ``examples/meta_learning/protonet_omniglot_pytorch`` (``model_def.py``
``OmniglotProtoNetTrial``: 4 x [conv3x3 - BatchNorm - ReLU - MaxPool2] embedding of 28x28 images,
N-way K-shot episodes, prototypes = mean support embedding, logits = -squared distance, Adam +
StepLR(reduce_every, lr_gamma) stepped per epoch, a batch = several episodes averaged).  The
Omniglot images cannot be downloaded here: ``SyntheticGlyphTasks`` draws episodes from a fixed
pool of random stroke-like 28x28 "characters" (per-class template + per-sample jitter/noise), so
meta-training still learns an embedding that separates unseen classes.
"""
from typing import Any, Dict, List

import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.utils.data as tud

from determined_1_amd import pytorch as det_torch


class SyntheticGlyphTasks(tud.Dataset):
    """Episodes of ``n_way`` classes x (``k_shot`` support + ``n_query`` query) images drawn from
    the ``class_ids`` subset of a fixed pool of synthetic glyph classes."""

    def __init__(self, n_tasks: int, class_ids: List[int], n_way: int, k_shot: int, n_query: int,
                 size: int = 28, n_pool: int = 1200, seed: int = 0) -> None:
        self.n_tasks = n_tasks
        self.class_ids = list(class_ids)
        self.n_way, self.k_shot, self.n_query, self.size = n_way, k_shot, n_query, size
        g = torch.Generator().manual_seed(1234)  # the glyph pool is shared by all splits
        coarse = (torch.rand(n_pool, 1, 7, 7, generator=g) > 0.6).float()
        self.templates = F.interpolate(coarse, size=(size, size), mode="bilinear", align_corners=False)
        self.seed = seed

    def __len__(self) -> int:
        return self.n_tasks

    def _sample(self, cls: int, n: int, g: torch.Generator) -> torch.Tensor:
        t = self.templates[cls].expand(n, 1, self.size, self.size)
        shift = torch.randint(-2, 3, (2,), generator=g).tolist()
        x = torch.roll(t, shifts=(shift[0], shift[1]), dims=(2, 3))
        return (x + 0.3 * torch.randn(x.shape, generator=g)).clamp(0, 1)

    def __getitem__(self, i: int) -> Dict[str, Any]:
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        pick = torch.randperm(len(self.class_ids), generator=g)[:self.n_way].tolist()
        xs, ys, xq, yq = [], [], [], []
        for label, j in enumerate(pick):
            x = self._sample(self.class_ids[j], self.k_shot + self.n_query, g)
            xs.append(x[:self.k_shot])
            xq.append(x[self.k_shot:])
            ys += [label] * self.k_shot
            yq += [label] * self.n_query
        return {"support": (torch.cat(xs), torch.tensor(ys)), "query": (torch.cat(xq), torch.tensor(yq))}


def collate_tasks(batch: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
    return batch


def squared_distance(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    return (x.unsqueeze(1) - y.unsqueeze(0)).pow(2).sum(-1)


def conv_block(cin: int, cout: int) -> nn.Module:
    return nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(), nn.MaxPool2d(2))
