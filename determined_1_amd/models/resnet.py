"""ResNet family (He et al. 2015, v1.5: stride on the 3x3 conv of the bottleneck), the
architecture of the north-star benchmark (ResNet-50, 224x224x3, 1000 classes).

Written for MI355X training: the model is meant to run in ``channels_last`` (NHWC) memory
format, which is the layout MIOpen's fastest bf16 convolution/batch-norm kernels consume on
gfx950, and the input pipeline kernel (``ops.u8_normalize``) produces NHWC directly.
``zero_init_residual`` zeroes the last BN gamma of each block (standard large-batch recipe).
"""
import threading
from typing import List, Optional, Type, Union

import torch
import torch.nn as nn

from determined_1_amd.ops import conv as native_conv
from determined_1_amd.ops.norm import BatchNormAct2d, linked_conv2d
from determined_1_amd.ops.pool import MaxPool3x3s2, global_avg_pool

# Fused BN(+add)(+ReLU) HIP kernels (ops/csrc/det_norm.hip) on by default; set
# ``resnet.FUSED_BN = False`` (or hparam ``fused_bn: false``) for the stock MIOpen path.
FUSED_BN = True
# Stride-1 1x1 convs as hand-written MFMA GEMMs with the BN statistics in the forward epilogue
# (ops/csrc/det_conv.hip); hparam ``native_conv1x1: false`` keeps them on MIOpen (A/B).
NATIVE_CONV1X1 = True

# Deferred BN forward applies (ops.conv DEFER_FWD_APPLY) hand the NEXT block an unwritten output
# buffer that its conv1 fills while staging its GEMM operand.  Only this file's own code may see such
# a buffer, so a block defers only inside ResNet.forward (blocks called one by one from user code
# never do) and only while no forward hook, forward pre-hook of its successor, or global module hook
# could observe the intermediate output (feature extraction, activation statistics, TensorBoard
# histogram callbacks).
_FWD = threading.local()


def _unobserved(block: nn.Module, nxt: Optional[nn.Module]) -> bool:
    from torch.nn.modules import module as _m

    if block._forward_hooks or _m._global_forward_hooks or _m._global_forward_pre_hooks:
        return False
    return nxt is None or not (nxt._forward_pre_hooks or nxt._forward_hooks)
# Bottleneck bn2 applied inside conv3's GEMM prologue (stats-only BN pass, no normalised
# activation in HBM).  Off by default: measured 1.1 % slower end to end on the MI355X (9,949 vs
# 10,056 samples/s, profiles/r2_bench_resnet50_bn_prologue_ab.jsonl) -- the prologue's VALU work
# in the forward and wgrad GEMMs costs more than the two activation passes it saves.
BN_PROLOGUE = False
# 7x7/2 stem conv as an implicit GEMM on the det_conv MFMA tiles with the stem BN's statistics in
# its epilogue (ops.conv.stem_conv; input channels padded to 4); hparam ``native_stem: false``
# keeps it on MIOpen (A/B).
NATIVE_STEM = True
# 3x3 convs on the det_igemm implicit GEMM (forward with the BN statistics in its epilogue, stride-1
# input gradient through the flipped weight, im2col weight gradient; ops.conv.conv_rs); hparam
# ``native_conv3x3: false`` keeps them on MIOpen (A/B).
NATIVE_CONV3X3 = True


def c3x3(x: torch.Tensor, conv: nn.Conv2d, bn_exclusive: bool = False) -> torch.Tensor:
    if NATIVE_CONV3X3 and FUSED_BN:
        return native_conv.conv_rs(x, conv, bn_exclusive=bn_exclusive)
    return conv(x)


def c1x1(x: torch.Tensor, conv: nn.Conv2d, bn_exclusive: bool = False) -> torch.Tensor:
    if NATIVE_CONV1X1 and FUSED_BN:
        return native_conv.conv1x1(x, conv, bn_exclusive=bn_exclusive)
    native_conv.materialize_fwd_apply(x)  # a deferred bn3 apply of the previous block
    return conv(x)


def bn_relu_c1x1(x: torch.Tensor, bn_mod: BatchNormAct2d, conv: nn.Conv2d) -> torch.Tensor:
    """``conv(relu(bn(x)))`` with the BN applied in the 1x1 GEMM's A-operand prologue (the normalised
    activation is never written to HBM; ``ops.conv.bn_relu_conv1x1``)."""
    if NATIVE_CONV1X1 and FUSED_BN and BN_PROLOGUE:
        return native_conv.bn_relu_conv1x1(x, bn_mod, conv)
    return c1x1(bn_mod(x), conv, bn_exclusive=True)  # bn2's output feeds only conv3


def bn(c: int, relu: bool) -> BatchNormAct2d:
    return BatchNormAct2d(c, relu=relu, fused=FUSED_BN)


def conv3x3(cin: int, cout: int, stride: int = 1, groups: int = 1, dilation: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=dilation, groups=groups, bias=False, dilation=dilation)


def conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


def _shortcut_linked(downsample: Optional[nn.Module], x: torch.Tensor) -> bool:
    """True when ``x``'s shortcut consumer hands its gradient through the BN link, not autograd."""
    from determined_1_amd.ops import norm as _norm

    if not _norm.SHORTCUT_LINK:
        return False
    if downsample is None:
        return True  # identity: bn3(..., idt, shortcut_link=True)
    return (isinstance(downsample, nn.Sequential) and len(downsample) == 2
            and isinstance(downsample[0], nn.Conv2d) and isinstance(downsample[1], BatchNormAct2d))


def _quiet(mod: nn.Module) -> bool:
    """No forward hook anywhere on ``mod`` (or a global one) could observe an intermediate output."""
    from torch.nn.modules import module as _m

    if _m._global_forward_hooks or _m._global_forward_pre_hooks:
        return False
    return not any(m._forward_hooks or m._forward_pre_hooks for m in mod.modules())


def _shortcut(downsample: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """Projection shortcut; its conv's input gradient is summed inside the producer's fused BN
    backward (``linked_conv2d``) rather than added to conv1's input gradient by autograd.  Inside
    ResNet.forward (the block's residual BN is then its only reader) the shortcut BN's apply is
    deferred into that residual apply (ops.conv DEFER_AFFINE_APPLY)."""
    if (FUSED_BN and isinstance(downsample, nn.Sequential) and len(downsample) == 2
            and isinstance(downsample[0], nn.Conv2d) and isinstance(downsample[1], BatchNormAct2d)):
        defer = getattr(_FWD, "depth", 0) > 0 and _quiet(downsample)
        return downsample[1](linked_conv2d(x, downsample[0]), defer_affine=defer)
    return downsample(x)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None) -> None:
        super().__init__()
        self.conv1 = conv3x3(cin, planes, stride)
        self.bn1 = bn(planes, relu=True)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = bn(planes, relu=True)  # relu(bn2(conv2) + identity), fused
        self.downsample = downsample

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        idt = x if self.downsample is None else _shortcut(self.downsample, x)
        out = self.bn1(c3x3(x, self.conv1))
        return self.bn2(c3x3(out, self.conv2), idt, shortcut_link=self.downsample is None)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None) -> None:
        super().__init__()
        self.conv1 = conv1x1(cin, planes)
        self.bn1 = bn(planes, relu=True)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = bn(planes, relu=True)
        self.conv3 = conv1x1(planes, planes * self.expansion)
        self.bn3 = bn(planes * self.expansion, relu=True)  # relu(bn3(conv3) + identity), fused
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        # set by ResNet when the next block is an identity-shortcut Bottleneck, whose conv1 is the
        # first reader of this block's output and stages bn3's apply itself (ops.conv DEFER_FWD_APPLY)
        self.defer_out = False
        self._defer_next: List[nn.Module] = []  # [successor block] (a list: not registered as a submodule)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # x (the previous block's output) reaches autograd only through conv1: the shortcut's
        # gradient is handed to its producer through the BN link (identity or projection)
        out = self.bn1(c1x1(x, self.conv1, bn_exclusive=FUSED_BN and _shortcut_linked(self.downsample, x)))
        out = bn_relu_c1x1(c3x3(out, self.conv2, bn_exclusive=True), self.bn2, self.conv3)  # bn1 feeds only conv2
        # the projection runs after the main branch: autograd then runs its backward first (later
        # nodes go first among ready ones), so its input gradient is linked before conv1's dgrad,
        # whose epilogue sums it into the producer's BN-backward partials
        idt = x if self.downsample is None else _shortcut(self.downsample, x)
        # identity shortcut: its gradient goes straight to the previous block's fused BN backward
        defer = (self.defer_out and NATIVE_CONV1X1 and FUSED_BN and getattr(_FWD, "depth", 0) > 0
                 and _unobserved(self, self._defer_next[0] if self._defer_next else None))
        return self.bn3(out, idt, shortcut_link=self.downsample is None, defer_apply=defer)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int], num_classes: int = 1000,
                 zero_init_residual: bool = True) -> None:
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = bn(64, relu=True)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = MaxPool3x3s2() if FUSED_BN else nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _make_layer(self, block: Type[Union[BasicBlock, Bottleneck]], planes: int, blocks: int,
                    stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       bn(planes * block.expansion, relu=False))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        for blk, nxt in zip(layers[:-1], layers[1:]):  # identity-shortcut successor: conv1 reads first
            if isinstance(blk, Bottleneck) and isinstance(nxt, Bottleneck) and nxt.downsample is None:
                blk.defer_out = True
                blk._defer_next = [nxt]
        return nn.Sequential(*layers)

    def _stem(self, x: torch.Tensor) -> torch.Tensor:
        """conv1 on 3-channel images, or 4-channel ones with a zero 4th channel (``u8_normalize(pad4=True)``)."""
        if NATIVE_STEM and FUSED_BN:
            return native_conv.stem_conv(x, self.conv1, stats=self.bn1.training)
        return self.conv1(x[:, :3] if x.shape[1] == 4 and self.conv1.in_channels == 3 else x)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        _FWD.depth = getattr(_FWD, "depth", 0) + 1  # blocks may defer their output applies (see _FWD)
        try:
            # the stem BN's output feeds only the pool: the pool applies it (forward) and writes its
            # backward partials, unless a hook could observe that activation
            pool_fused = isinstance(self.maxpool, MaxPool3x3s2)
            x = self.bn1(self._stem(x), defer_affine=pool_fused and _quiet(self.bn1) and _quiet(self.maxpool))
            x = self.maxpool(x, bn_exclusive=True) if pool_fused else self.maxpool(x)
            x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        finally:
            _FWD.depth -= 1
        # the head's pooling on det_pool.hip (one read of the layer-4 output, one channels_last write
        # of its gradient) unless a hook could observe the pool module's output
        x = global_avg_pool(x) if FUSED_BN and _quiet(self.avgpool) else torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


def resnet18(**kw) -> ResNet:  # type: ignore
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw) -> ResNet:  # type: ignore
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw) -> ResNet:  # type: ignore
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw) -> ResNet:  # type: ignore
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)


def resnet152(**kw) -> ResNet:  # type: ignore
    return ResNet(Bottleneck, [3, 8, 36, 3], **kw)
