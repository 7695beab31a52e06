"""Localise a BN-backward-fusion mismatch: ResNet-50 grads with the fusion per mode vs off,
printed in backward order (deepest layers first)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from determined_1_amd.models import resnet  # noqa: E402
from determined_1_amd.ops import conv  # noqa: E402

gpu = torch.device("cuda")


def run(fuse, modes=(1, 2)):
    conv.FUSE_BN_BWD = fuse
    conv.FUSE_BN_BWD_MODES = modes
    torch.manual_seed(0)
    m = resnet.resnet50(num_classes=10, zero_init_residual=False).to(gpu).to(memory_format=torch.channels_last).to(torch.bfloat16)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.float()
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(4, 3, 64, 64, generator=g).to(gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (4,), generator=g).to(gpu)
    loss = torch.nn.functional.cross_entropy(m(conv.pad_channels4(x)).float(), y)
    loss.backward()
    return {n: p.grad.float().clone() for n, p in m.named_parameters()}


ref = run(False)
for modes in [(1,), (2,), (1, 2)]:
    got = run(True, modes)
    print("modes", modes, conv.BN_BWD_COUNTS)
    bad = 0
    for n in reversed(list(ref)):
        a, b = got[n], ref[n]
        rel = float((a - b).abs().max()) / (float(b.abs().max()) + 1e-6)
        if rel > 0.05:
            print(f"  {n}: rel {rel:.3f}")
            bad += 1
            if bad > 6:
                break
    print("  bad", bad)
