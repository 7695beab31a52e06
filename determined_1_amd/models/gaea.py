"""GAEA neural architecture search: weight-sharing search on CIFAR-10 and ImageNet evaluation.

Mirrors the reference's ``examples/nas/gaea_pytorch``:
  * ``search/`` (``model_def.py:34-159`` ``GAEASearchTrial``, ``model_search.py``,
    ``optimizer.py`` ``EG``, ``data.py`` ``BilevelDataset``): a PC-DARTS style supernet (every
    edge is a mixture of the 8 DARTS primitives applied to 1/``shuffle_factor`` of the channels,
    followed by a channel shuffle; per-edge weights ``betas`` normalise the inputs of each node)
    trained bilevel within ONE ``train_batch``: an SGD step of the shared weights on a train
    image batch, then an exponentiated-gradient (GAEA) step of the architecture weights on a
    held-out batch.  The two optimizers are two ``wrap_optimizer`` calls with two
    ``context.backward`` / ``step_optimizer`` pairs per batch.  The derived genotype is logged at
    every validation.
  * ``eval/`` (``model_def.py:48-268`` ``GAEAEvalTrial``, ``model.py`` ``NetworkImageNet``,
    ``utils.py``, ``lr_schedulers.py``): the searched cell stacked into an ImageNet network with
    swish activations, squeeze-and-excitation after the first 2/3 of the cells, Dropout2d before
    conv ops, drop-path, label smoothing, an exponential moving average of the weights evaluated
    alongside the live weights, and warmup + linear / cosine / EfficientNet LR schedules.
CIFAR-10 / ImageNet cannot be downloaded here: ``SyntheticClassification`` of those shapes
stands in (the reference's own eval ``const.yaml`` also runs on random data).

MI355X notes: the EMA update is one multi-tensor ``_foreach_lerp_`` launch over all weights (not a
per-tensor Python loop), the EG step is two fused in-place passes per architecture tensor, and the
architecture mixture weights are computed once per forward for all cells of a type.
"""
import logging
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_1_amd import pytorch as det_torch
from determined_1_amd.models.darts import OPS, PRIMITIVES, FactorizedReduce, ReLUConvBN, drop_path, topk_accuracy
from determined_1_amd.models.synthetic import SyntheticClassification


# ------------------------------------------------------------------------------------------------
# search
# ------------------------------------------------------------------------------------------------
def channel_shuffle(x: torch.Tensor, groups: int) -> torch.Tensor:
    n, c, h, w = x.shape
    return x.view(n, groups, c // groups, h, w).transpose(1, 2).reshape(n, c, h, w)


class MixedOp(nn.Module):
    """Partial-channel mixture: the primitives see the first C/k channels; the rest bypass
    (max-pooled on reduction edges); the result is channel-shuffled (reference
    ``model_search.py:25-51``)."""

    def __init__(self, c: int, stride: int, k: int) -> None:
        super().__init__()
        self.k = k
        self.ops = nn.ModuleList()
        for prim in PRIMITIVES:
            op = OPS[prim](c // k, stride, False)
            if "pool" in prim:
                op = nn.Sequential(op, nn.BatchNorm2d(c // k, affine=False))
            self.ops.append(op)
        self.bypass_pool = nn.MaxPool2d(2, 2)

    def forward(self, x: torch.Tensor, weights: torch.Tensor) -> torch.Tensor:
        part = x.shape[1] // self.k
        active, rest = x[:, :part], x[:, part:]
        mixed = sum(w * op(active) for w, op in zip(weights.unbind(0), self.ops))
        if mixed.shape[2] != x.shape[2]:
            rest = self.bypass_pool(rest)
        return channel_shuffle(torch.cat([mixed, rest], dim=1), self.k)


class SearchCell(nn.Module):
    def __init__(self, steps: int, multiplier: int, c_pp: int, c_p: int, c: int, reduction: bool,
                 reduction_prev: bool, k: int) -> None:
        super().__init__()
        self.reduction = reduction
        self.pre0 = FactorizedReduce(c_pp, c, affine=False) if reduction_prev else ReLUConvBN(c_pp, c, 1, 1, 0, False)
        self.pre1 = ReLUConvBN(c_p, c, 1, 1, 0, False)
        self.steps, self.multiplier = steps, multiplier
        self.edges = nn.ModuleList(MixedOp(c, 2 if reduction and j < 2 else 1, k)
                                   for i in range(steps) for j in range(2 + i))

    def forward(self, s0: torch.Tensor, s1: torch.Tensor, alphas: torch.Tensor, betas: torch.Tensor) -> torch.Tensor:
        states = [self.pre0(s0), self.pre1(s1)]
        off = 0
        for _ in range(self.steps):
            s = sum(betas[off + j] * self.edges[off + j](h, alphas[off + j]) for j, h in enumerate(states))
            off += len(states)
            states.append(s)
        return torch.cat(states[-self.multiplier:], dim=1)


def _edge_softmax(betas: torch.Tensor, steps: int) -> torch.Tensor:
    """Softmax of the edge weights over the inputs of each node (2, 3, 4, ... inputs)."""
    out, start = [], 0
    for i in range(steps):
        n = 2 + i
        out.append(F.softmax(betas[start:start + n], dim=-1))
        start += n
    return torch.cat(out)


class SearchNetwork(nn.Module):
    """Weight-sharing supernet (reference ``model_search.py:94-264``)."""

    def __init__(self, c: int, num_classes: int, layers: int, steps: int = 4, multiplier: Optional[int] = None,
                 stem_multiplier: int = 3, k: int = 4) -> None:
        super().__init__()
        multiplier = steps if multiplier is None else multiplier  # the cell concatenates its last nodes
        self.steps, self.multiplier = steps, multiplier
        c_cur = stem_multiplier * c
        self.stem = nn.Sequential(nn.Conv2d(3, c_cur, 3, padding=1, bias=False), nn.BatchNorm2d(c_cur))
        c_pp, c_p, c_cur = c_cur, c_cur, c
        self.cells = nn.ModuleList()
        reduction_prev = False
        for i in range(layers):
            reduction = i in (layers // 3, 2 * layers // 3)
            if reduction:
                c_cur *= 2
            self.cells.append(SearchCell(steps, multiplier, c_pp, c_p, c_cur, reduction, reduction_prev, k))
            reduction_prev = reduction
            c_pp, c_p = c_p, multiplier * c_cur
        self.classifier = nn.Linear(c_p, num_classes)
        self._ws = list(self.parameters())
        n_edges = sum(2 + i for i in range(steps))
        self.alphas_normal = nn.Parameter(torch.ones(n_edges, len(PRIMITIVES)))
        self.alphas_reduce = nn.Parameter(torch.ones(n_edges, len(PRIMITIVES)))
        self.betas_normal = nn.Parameter(torch.ones(n_edges))
        self.betas_reduce = nn.Parameter(torch.ones(n_edges))

    def ws_parameters(self) -> List[nn.Parameter]:
        return self._ws

    def arch_parameters(self) -> List[nn.Parameter]:
        return [self.alphas_normal, self.alphas_reduce, self.betas_normal, self.betas_reduce]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        w = {False: (F.softmax(self.alphas_normal, dim=-1), _edge_softmax(self.betas_normal, self.steps)),
             True: (F.softmax(self.alphas_reduce, dim=-1), _edge_softmax(self.betas_reduce, self.steps))}
        s0 = s1 = self.stem(x)
        for cell in self.cells:
            a, b = w[cell.reduction]
            s0, s1 = s1, cell(s0, s1, a, b)
        return self.classifier(F.adaptive_avg_pool2d(s1, 1).flatten(1))

    def genotype(self) -> Dict[str, Any]:
        """Top-2 incoming edges per node by their strongest non-``none`` op weight (scaled by the
        edge weight), each with its best non-``none`` op (reference ``model_search.py:204-264``)."""
        none = PRIMITIVES.index("none")

        def parse(alphas: torch.Tensor, betas: torch.Tensor) -> List[Tuple[str, int]]:
            W = (F.softmax(alphas, dim=-1) * _edge_softmax(betas, self.steps)[:, None]).detach().cpu()
            W[:, none] = -1.0
            gene, start = [], 0
            for i in range(self.steps):
                n = 2 + i
                block = W[start:start + n]
                best = block.max(dim=1)
                for j in sorted(range(n), key=lambda e: -float(best.values[e]))[:2]:
                    gene.append((PRIMITIVES[int(best.indices[j])], j))
                start += n
            return gene

        concat = list(range(2 + self.steps - self.multiplier, self.steps + 2))
        return {"normal": parse(self.alphas_normal, self.betas_normal), "normal_concat": concat,
                "reduce": parse(self.alphas_reduce, self.betas_reduce), "reduce_concat": concat}


class EG(torch.optim.Optimizer):
    """Exponentiated gradient on the simplex: p <- p * exp(-lr * g), then renormalised along the
    last dim (reference ``search/optimizer.py``; the GAEA update)."""

    def __init__(self, params: Any, lr: float) -> None:
        if lr < 0:
            raise ValueError(f"invalid learning rate {lr}")
        super().__init__(params, dict(lr=lr))

    @torch.no_grad()
    def step(self, closure: Any = None) -> Any:
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is None:
                    continue
                p.mul_(torch.exp(p.grad * -g["lr"]))
                p.div_(p.sum(dim=-1, keepdim=True))
        return loss


class BilevelPairs(torch.utils.data.Dataset):
    """Each item pairs a sample of the first half of ``dataset`` (shared-weight step) with one of
    the second half (architecture step); the pairing is reshuffled every epoch (reference
    ``search/data.py``)."""

    def __init__(self, dataset: torch.utils.data.Dataset, seed: int = 0) -> None:
        self.dataset = dataset
        n = len(dataset) // 2  # type: ignore
        self.train_idx = list(range(n))
        self.val_idx = list(range(n, 2 * n))
        self.gen = torch.Generator().manual_seed(seed)

    def shuffle_val(self) -> None:
        perm = torch.randperm(len(self.val_idx), generator=self.gen).tolist()
        self.val_idx = [self.val_idx[i] for i in perm]

    def __len__(self) -> int:
        return len(self.train_idx)

    def __getitem__(self, i: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
        xt, yt = self.dataset[self.train_idx[i]]
        xv, yv = self.dataset[self.val_idx[i]]
        return xt, yt, xv, yv


GAEA_IMAGENET_GENOTYPE = {
    "normal": [("skip_connect", 1), ("skip_connect", 0), ("sep_conv_3x3", 2), ("sep_conv_3x3", 1),
               ("sep_conv_5x5", 2), ("sep_conv_3x3", 0), ("sep_conv_5x5", 3), ("sep_conv_5x5", 2)],
    "normal_concat": [2, 3, 4, 5],
    "reduce": [("max_pool_3x3", 1), ("sep_conv_3x3", 0), ("sep_conv_5x5", 1), ("dil_conv_5x5", 2),
               ("sep_conv_3x3", 1), ("sep_conv_3x3", 3), ("sep_conv_5x5", 1), ("max_pool_3x3", 2)],
    "reduce_concat": [2, 3, 4, 5],
}  # reference eval/model_def.py:75-98

ACTIVATIONS = {"relu": nn.ReLU, "swish": nn.SiLU, "hswish": nn.Hardswish}


class SqueezeExcite(nn.Module):
    def __init__(self, c: int, hidden: int, act: Callable[[], nn.Module]) -> None:
        super().__init__()
        self.reduce = nn.Conv2d(c, hidden, 1)
        self.expand = nn.Conv2d(hidden, c, 1)
        self.act = act()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x * torch.sigmoid(self.expand(self.act(self.reduce(x.mean((2, 3), keepdim=True)))))


class EvalCell(nn.Module):
    def __init__(self, genotype: Dict[str, Any], c_pp: int, c_p: int, c: int, reduction: bool, reduction_prev: bool,
                 act: Callable[[], nn.Module], drop_prob: float) -> None:
        super().__init__()
        self.pre0 = FactorizedReduce(c_pp, c, act=act) if reduction_prev else ReLUConvBN(c_pp, c, 1, 1, 0, act=act)
        self.pre1 = ReLUConvBN(c_p, c, 1, 1, 0, act=act)
        edges = genotype["reduce" if reduction else "normal"]
        self.concat = list(genotype["reduce_concat" if reduction else "normal_concat"])
        self.multiplier = len(self.concat)
        self.ops = nn.ModuleList()
        self.inputs = []  # type: List[int]
        for name, idx in edges:
            op = OPS[name](c, 2 if reduction and idx < 2 else 1, True, act)
            if "conv" in name and drop_prob > 0:
                op = nn.Sequential(nn.Dropout2d(drop_prob), op)
            self.ops.append(op)
            self.inputs.append(int(idx))

    def forward(self, s0: torch.Tensor, s1: torch.Tensor, p_drop: float) -> torch.Tensor:
        states = [self.pre0(s0), self.pre1(s1)]
        for i in range(len(self.ops) // 2):
            hs = []
            for e in (2 * i, 2 * i + 1):
                h = self.ops[e](states[self.inputs[e]])
                if self.training and p_drop > 0 and not isinstance(self.ops[e], nn.Identity):
                    h = drop_path(h, p_drop)
                hs.append(h)
            states.append(hs[0] + hs[1])
        return torch.cat([states[i] for i in self.concat], dim=1)


class NetworkImageNet(nn.Module):
    """Reference ``eval/model.py:108-209``: two stride-2 stems + stride-2 stem1 (224 -> 28),
    cells with reductions at 1/3 and 2/3 depth, SE on the first 2/3, optional auxiliary head."""

    def __init__(self, genotype: Dict[str, Any], act: Callable[[], nn.Module], c: int, num_classes: int, layers: int,
                 auxiliary: bool, do_se: bool, drop_path_prob: float = 0.0, drop_prob: float = 0.0) -> None:
        super().__init__()
        self.layers, self.do_se, self.drop_path_prob = layers, do_se, drop_path_prob
        # the reference passes the TF-style decay 0.999 as torch's `momentum` (which would weight the
        # newest batch by 0.999); the intended TF semantics are torch momentum 0.001
        bn = dict(momentum=0.001, eps=1e-3)
        self.stem0 = nn.Sequential(nn.Conv2d(3, c // 2, 3, 2, 1, bias=False), nn.BatchNorm2d(c // 2, **bn), act(),
                                   nn.Conv2d(c // 2, c, 3, 2, 1, bias=False), nn.BatchNorm2d(c, **bn))
        self.stem1 = nn.Sequential(act(), nn.Conv2d(c, c, 3, 2, 1, bias=False), nn.BatchNorm2d(c, **bn))
        c_pp, c_p, c_cur = c, c, c
        self.cells = nn.ModuleList()
        self.se = nn.ModuleList()
        reduction_prev = True
        c_aux = c_p
        for i in range(layers):
            reduction = i in (layers // 3, 2 * layers // 3)
            if reduction:
                c_cur *= 2
            cell = EvalCell(genotype, c_pp, c_p, c_cur, reduction, reduction_prev, act, drop_prob)
            reduction_prev = reduction
            self.cells.append(cell)
            c_pp, c_p = c_p, cell.multiplier * c_cur
            if do_se and i <= layers * 2 / 3:
                self.se.append(SqueezeExcite(c_cur * 4, c_cur // (4 if c_cur == c else 8), act))
            if i == 2 * layers // 3:
                c_aux = c_p
        self.aux = None  # type: Optional[nn.Module]
        if auxiliary:
            self.aux = nn.Sequential(act(), nn.AvgPool2d(5, 2, 0, count_include_pad=False),
                                     nn.Conv2d(c_aux, 128, 1, bias=False), nn.BatchNorm2d(128, **bn), act(),
                                     nn.Conv2d(128, 768, 2, bias=False), nn.BatchNorm2d(768, **bn), act(),
                                     nn.Flatten(), nn.Linear(768, num_classes))
        self.classifier = nn.Linear(c_p, num_classes)

    def forward(self, x: torch.Tensor) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        logits_aux = None
        s0 = self.stem0(x)
        s1 = self.stem1(s0)
        for i, cell in enumerate(self.cells):
            s0, s1 = s1, cell(s0, s1, self.drop_path_prob)
            if self.do_se and i <= len(self.cells) * 2 / 3:
                s1 = self.se[i](s1)
            if i == 2 * self.layers // 3 and self.aux is not None and self.training:
                logits_aux = self.aux(s1)
        return self.classifier(F.adaptive_avg_pool2d(s1, 1).flatten(1)), logits_aux


class EMAModel(nn.Module):
    """Wraps a model with an exponential moving average of its parameters and floating-point
    buffers (reference ``eval/utils.py:15-76`` ``EMAWrapper``).  The shadow copies are buffers,
    so they are checkpointed and broadcast with the model.  ``swap()`` exchanges live and averaged
    weights in place (call twice to restore)."""

    def __init__(self, model: nn.Module, decay: float) -> None:
        super().__init__()
        self.model = model
        self.decay = decay
        for i, t in enumerate(self._tracked()):
            self.register_buffer(f"ema_{i}", t.detach().clone())

    def _tracked(self) -> List[torch.Tensor]:
        ts = [p.data for p in self.model.parameters()]
        ts += [b for b in self.model.buffers() if b.is_floating_point()]
        return ts

    def _shadow(self) -> List[torch.Tensor]:
        return [b for n, b in self.named_buffers(recurse=False) if n.startswith("ema_")]

    def forward(self, *args: Any) -> Any:
        return self.model(*args)

    @torch.no_grad()
    def update(self) -> None:
        torch._foreach_lerp_(self._shadow(), self._tracked(), 1.0 - self.decay)

    @torch.no_grad()
    def swap(self) -> None:
        for live, shadow in zip(self._tracked(), self._shadow()):
            tmp = live.clone()
            live.copy_(shadow)
            shadow.copy_(tmp)


def label_smoothing_ce(logits: torch.Tensor, target: torch.Tensor, eps: float) -> torch.Tensor:
    """Reference ``CrossEntropyLabelSmooth``: (1-eps) * one_hot + eps / K targets."""
    return F.cross_entropy(logits, target, label_smoothing=eps)


def lr_multiplier(kind: str, epoch: int, warmup: int, max_epochs: int, gamma: float = 0.97,
                  decay_every: int = 2) -> float:
    """Warmup + {linear, cosine, efficientnet} (reference ``eval/lr_schedulers.py``)."""
    import math

    if epoch < warmup:
        return (epoch + 1) / warmup
    if kind == "linear":
        if max_epochs - epoch > warmup:
            return (max_epochs - warmup - epoch) / (max_epochs - warmup)
        return (max_epochs - epoch) / ((epoch - warmup) * 5)
    if kind == "cosine":
        return 0.5 * (1 + math.cos(math.pi * epoch / max_epochs))
    if kind == "efficientnet":
        return gamma ** int((epoch + 1) / decay_every)
    raise ValueError(f"unknown lr_scheduler {kind!r}")
