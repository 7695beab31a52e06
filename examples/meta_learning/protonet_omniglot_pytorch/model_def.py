"""Prototypical-network few-shot trial (reference examples/meta_learning/protonet_omniglot_pytorch):
the networks and helpers come from the ``determined_1_amd.models.protonet`` library  Synthetic glyph episodes stand in for Omniglot.

This file is the experiment's user code (it is what a checkpoint's ``code/`` holds): the
Trial -- data, optimizer, training and evaluation steps -- lives here; the network building
blocks are imported from the framework's model library, as the reference examples import theirs
from torchvision / transformers.
"""
from typing import Any, Dict, List

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_1_amd import pytorch as det_torch
from determined_1_amd.models.protonet import SyntheticGlyphTasks, collate_tasks, conv_block, squared_distance


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



OmniglotProtoNetTrial = ProtoNetTrial  # the reference example's class name
