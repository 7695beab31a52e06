"""DARTS CIFAR-10 network trained from a hyperparameter-encoded genotype.

Mirrors the reference's ``examples/hp_search_benchmarks/darts_cifar10_pytorch`` (``DARTSCNNTrial``):
the architecture search space of DARTS (Liu et al. 2019) is exposed as hyperparameters — for each
of the 4 intermediate nodes of the normal and the reduction cell, two input edges
(``{cell}_node{i}_edge{j}`` = index of the input state) and their operations
(``{cell}_node{i}_edge{j}_op``) — so Determined's searchers (``adaptive.yaml``: adaptive ASHA over
those categoricals) perform the NAS.  Training follows the DARTS evaluation protocol: SGD-momentum,
cosine annealing per epoch, drop-path probability ramped linearly over ``train_epochs``, auxiliary
head at 2/3 depth (weight ``auxiliary_weight``), gradient clipping at ``clip_gradients_l2_norm``.
CIFAR-10 cannot be downloaded here: ``SyntheticClassification`` of the CIFAR shape stands in.

The operations are the standard DARTS primitives, written for channels_last bf16 execution on
MI355X (MIOpen depthwise/pointwise convolutions).
"""
from typing import Any, Callable, Dict, List, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_1_amd import pytorch as det_torch
from determined_1_amd.models.synthetic import SyntheticClassification

PRIMITIVES = ("none", "max_pool_3x3", "avg_pool_3x3", "skip_connect", "sep_conv_3x3", "sep_conv_5x5",
              "dil_conv_3x3", "dil_conv_5x5")


class ReLUConvBN(nn.Sequential):
    """act -> conv -> BN (``act`` is ReLU in DARTS, swish in the GAEA ImageNet network)."""

    def __init__(self, cin: int, cout: int, k: int, stride: int, pad: int, affine: bool = True,
                 act: Callable[[], nn.Module] = nn.ReLU) -> None:
        super().__init__(act(), nn.Conv2d(cin, cout, k, stride, pad, bias=False), nn.BatchNorm2d(cout, affine=affine))


class DilConv(nn.Sequential):
    """ReLU -> depthwise k x k (dilation d) -> pointwise 1x1 -> BN."""

    def __init__(self, cin: int, cout: int, k: int, stride: int, pad: int, dilation: int, affine: bool = True,
                 act: Callable[[], nn.Module] = nn.ReLU) -> None:
        super().__init__(act(),
                         nn.Conv2d(cin, cin, k, stride, pad, dilation=dilation, groups=cin, bias=False),
                         nn.Conv2d(cin, cout, 1, bias=False), nn.BatchNorm2d(cout, affine=affine))


class SepConv(nn.Sequential):
    """Two stacked dilation-1 DilConv blocks, the first carrying the stride."""

    def __init__(self, cin: int, cout: int, k: int, stride: int, pad: int, affine: bool = True,
                 act: Callable[[], nn.Module] = nn.ReLU) -> None:
        super().__init__(DilConv(cin, cin, k, stride, pad, 1, affine, act), DilConv(cin, cout, k, 1, pad, 1, affine, act))


class Zero(nn.Module):
    def __init__(self, stride: int) -> None:
        super().__init__()
        self.stride = stride

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x[:, :, ::self.stride, ::self.stride] * 0.0


class FactorizedReduce(nn.Module):
    """Stride-2 1x1 convolutions on two offset pixel grids, concatenated (shape-preserving skip)."""

    def __init__(self, cin: int, cout: int, affine: bool = True, act: Callable[[], nn.Module] = nn.ReLU) -> None:
        super().__init__()
        self.act = act()
        self.conv1 = nn.Conv2d(cin, cout // 2, 1, 2, bias=False)
        self.conv2 = nn.Conv2d(cin, cout - cout // 2, 1, 2, bias=False)
        self.bn = nn.BatchNorm2d(cout, affine=affine)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.act(x)
        return self.bn(torch.cat([self.conv1(x), self.conv2(x[:, :, 1:, 1:])], dim=1))


OPS = {
    "none": lambda c, s, affine=True, act=nn.ReLU: Zero(s),
    "max_pool_3x3": lambda c, s, affine=True, act=nn.ReLU: nn.MaxPool2d(3, s, 1),
    "avg_pool_3x3": lambda c, s, affine=True, act=nn.ReLU: nn.AvgPool2d(3, s, 1, count_include_pad=False),
    "skip_connect": lambda c, s, affine=True, act=nn.ReLU: nn.Identity() if s == 1 else FactorizedReduce(c, c, affine, act),
    "sep_conv_3x3": lambda c, s, affine=True, act=nn.ReLU: SepConv(c, c, 3, s, 1, affine, act),
    "sep_conv_5x5": lambda c, s, affine=True, act=nn.ReLU: SepConv(c, c, 5, s, 2, affine, act),
    "dil_conv_3x3": lambda c, s, affine=True, act=nn.ReLU: DilConv(c, c, 3, s, 2, 2, affine, act),
    "dil_conv_5x5": lambda c, s, affine=True, act=nn.ReLU: DilConv(c, c, 5, s, 4, 2, affine, act),
}  # type: Dict[str, Callable[..., nn.Module]]


def drop_path(x: torch.Tensor, p: float) -> torch.Tensor:
    keep = 1.0 - p
    mask = torch.empty(x.shape[0], 1, 1, 1, device=x.device, dtype=x.dtype).bernoulli_(keep)
    return x / keep * mask


class Cell(nn.Module):
    """4 intermediate nodes; node i sums two ops applied to earlier states (0, 1 = the two cell
    inputs); the cell output concatenates nodes 2..5 (all intermediates)."""

    def __init__(self, edges: Sequence[Tuple[str, int]], c_pp: int, c_p: int, c: int, reduction: bool,
                 reduction_prev: bool) -> None:
        super().__init__()
        self.pre0 = FactorizedReduce(c_pp, c) if reduction_prev else ReLUConvBN(c_pp, c, 1, 1, 0)
        self.pre1 = ReLUConvBN(c_p, c, 1, 1, 0)
        self.reduction = reduction
        self.ops = nn.ModuleList()
        self.inputs = []  # type: List[int]
        for name, idx in edges:
            stride = 2 if reduction and idx < 2 else 1
            self.ops.append(OPS[name](c, stride))
            self.inputs.append(int(idx))
        self.multiplier = 4

    def forward(self, s0: torch.Tensor, s1: torch.Tensor, p_drop: float) -> torch.Tensor:
        states = [self.pre0(s0), self.pre1(s1)]
        for node in range(4):
            total = None
            for e in (2 * node, 2 * node + 1):
                op = self.ops[e]
                h = op(states[self.inputs[e]])
                if self.training and p_drop > 0 and not isinstance(op, nn.Identity):
                    h = drop_path(h, p_drop)
                total = h if total is None else total + h
            states.append(total)
        return torch.cat(states[2:], dim=1)


class AuxiliaryHead(nn.Module):
    """DARTS CIFAR auxiliary classifier on 8x8 feature maps."""

    def __init__(self, c: int, num_classes: int) -> None:
        super().__init__()
        self.features = nn.Sequential(
            nn.ReLU(inplace=False), nn.AvgPool2d(5, stride=3, padding=0, count_include_pad=False),
            nn.Conv2d(c, 128, 1, bias=False), nn.BatchNorm2d(128), nn.ReLU(inplace=False),
            nn.Conv2d(128, 768, 2, bias=False), nn.BatchNorm2d(768), nn.ReLU(inplace=False))
        self.classifier = nn.Linear(768, num_classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.classifier(torch.flatten(self.features(x), 1))


class DARTSNetwork(nn.Module):
    def __init__(self, c: int, num_classes: int, layers: int, auxiliary: bool, normal: Sequence[Tuple[str, int]],
                 reduce: Sequence[Tuple[str, int]]) -> None:
        super().__init__()
        self.drop_path_prob = 0.0
        self.aux_at = 2 * layers // 3
        c_cur = 3 * c
        self.stem = nn.Sequential(nn.Conv2d(3, c_cur, 3, padding=1, bias=False), nn.BatchNorm2d(c_cur))
        c_pp, c_p, c_cur = c_cur, c_cur, c
        self.cells = nn.ModuleList()
        reduction_prev = False
        c_aux = 0
        for i in range(layers):
            reduction = i in (layers // 3, 2 * layers // 3)
            if reduction:
                c_cur *= 2
            cell = Cell(reduce if reduction else normal, c_pp, c_p, c_cur, reduction, reduction_prev)
            reduction_prev = reduction
            self.cells.append(cell)
            c_pp, c_p = c_p, cell.multiplier * c_cur
            if i == self.aux_at:
                c_aux = c_p
        self.aux = AuxiliaryHead(c_aux, num_classes) if auxiliary else None
        self.classifier = nn.Linear(c_p, num_classes)

    def forward(self, x: torch.Tensor) -> Tuple[torch.Tensor, Any]:
        s0 = s1 = self.stem(x)
        logits_aux = None
        for i, cell in enumerate(self.cells):
            s0, s1 = s1, cell(s0, s1, self.drop_path_prob)
            if i == self.aux_at and self.aux is not None and self.training:
                logits_aux = self.aux(s1)
        out = F.adaptive_avg_pool2d(s1, 1).flatten(1)
        return self.classifier(out), logits_aux


def genotype_from_hparams(hp: Dict[str, Any]) -> Dict[str, List[Tuple[str, int]]]:
    """``{cell}_node{i}_edge{j}`` / ``..._op`` hyperparameters -> (op, input state) per edge."""
    g = {"normal": [], "reduce": []}  # type: Dict[str, List[Tuple[str, int]]]
    for cell in ("normal", "reduce"):
        for node in range(1, 5):
            for edge in (1, 2):
                idx = int(hp[f"{cell}_node{node}_edge{edge}"])
                op = str(hp[f"{cell}_node{node}_edge{edge}_op"])
                if op not in OPS:
                    raise ValueError(f"{cell} node {node} edge {edge}: unknown op {op!r} (one of {PRIMITIVES})")
                if not 0 <= idx <= node:
                    raise ValueError(f"{cell} node {node} edge {edge}: input {idx} must be in [0, {node}]")
                g[cell].append((op, idx))
    return g


def topk_accuracy(logits: torch.Tensor, target: torch.Tensor, ks: Sequence[int] = (1, 5)) -> List[torch.Tensor]:
    top = logits.topk(max(ks), dim=1).indices
    hit = top == target[:, None]
    return [hit[:, :k].any(dim=1).float().mean() for k in ks]
