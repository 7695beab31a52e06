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


class ProtoNetTrial(det_torch.PyTorchTrial):
    def __init__(self, context: det_torch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        self.n_way = {"train": int(hp.get("num_classes_train", 60)), "val": int(hp.get("num_classes_val", 20))}
        self.k_shot = {"train": int(hp.get("num_support_train", 1)), "val": int(hp.get("num_support_val", 1))}
        self.n_query = {"train": int(hp.get("num_query_train", 5)), "val": int(hp.get("num_query_val", 5))}
        n_pool = int(hp.get("num_glyph_classes", 1200))
        n_val = int(n_pool * float(hp.get("validation_portion", 0.25)))
        perm = torch.randperm(n_pool, generator=torch.Generator().manual_seed(7)).tolist()
        self.val_classes, self.train_classes = perm[:n_val], perm[n_val:]
        hid, z = int(hp.get("hidden_dim", 64)), int(hp.get("embedding_dim", 64))
        self.model = context.wrap_model(nn.Sequential(conv_block(1, hid), conv_block(hid, hid), conv_block(hid, hid),
                                                      conv_block(hid, z), nn.Flatten()))
        self.opt = context.wrap_optimizer(torch.optim.Adam(self.model.parameters(),
                                                           lr=float(hp.get("learning_rate", 1e-3)),
                                                           weight_decay=float(hp.get("weight_decay", 0.0))))
        self.sched = context.wrap_lr_scheduler(
            torch.optim.lr_scheduler.StepLR(self.opt, int(hp.get("reduce_every", 200)), gamma=float(hp.get("lr_gamma", 0.5))),
            det_torch.LRScheduler.StepMode.STEP_EVERY_EPOCH)

    def episode_loss(self, task: Dict[str, Any], split: str):
        xs, ys = task["support"]
        xq, yq = task["query"]
        n, k = self.n_way[split], self.k_shot[split]
        emb = self.model(torch.cat([xs, xq], 0))
        # support is class-major (labels 0..n-1, k each): prototypes = per-class mean embedding
        protos = emb[:n * k].view(n, k, -1).mean(1)
        logits = -squared_distance(emb[n * k:], protos)
        loss = F.cross_entropy(logits, yq)
        acc = (logits.argmax(-1) == yq).float().mean()
        return loss, acc

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        losses, accs = zip(*(self.episode_loss(t, "train") for t in batch))
        loss = torch.stack(losses).mean()
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss, "acc": torch.stack(accs).mean()}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        losses, accs = zip(*(self.episode_loss(t, "val") for t in batch))
        return {"loss": torch.stack(losses).mean(), "acc": torch.stack(accs).mean()}

    def build_training_data_loader(self) -> det_torch.DataLoader:
        hp = self.context.get_hparams()
        ds = SyntheticGlyphTasks(int(hp.get("tasks_per_epoch_train", 100)), self.train_classes, self.n_way["train"],
                                 self.k_shot["train"], self.n_query["train"],
                                 n_pool=int(hp.get("num_glyph_classes", 1200)))
        return det_torch.DataLoader(ds, batch_size=self.context.get_per_slot_batch_size(), collate_fn=collate_tasks)

    def build_validation_data_loader(self) -> det_torch.DataLoader:
        hp = self.context.get_hparams()
        ds = SyntheticGlyphTasks(int(hp.get("tasks_per_epoch_val", 100)), self.val_classes, self.n_way["val"],
                                 self.k_shot["val"], self.n_query["val"], n_pool=int(hp.get("num_glyph_classes", 1200)),
                                 seed=1)
        return det_torch.DataLoader(ds, batch_size=int(hp.get("val_batch_size", 2)), collate_fn=collate_tasks)
