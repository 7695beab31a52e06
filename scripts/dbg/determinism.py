"""Is the ResNet-50 fwd/bwd deterministic run to run (same weights/data)?  Per native-path toggle."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from determined_1_amd.models import resnet  # noqa: E402
from determined_1_amd.ops import conv  # noqa: E402

gpu = torch.device("cuda")


def run(hw=64, bs=4):
    torch.manual_seed(0)
    m = resnet.resnet50(num_classes=10, zero_init_residual=False).to(gpu).to(memory_format=torch.channels_last).to(torch.bfloat16)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.float()
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(bs, 3, hw, hw, generator=g).to(gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (bs,), generator=g).to(gpu)
    out = m(conv.pad_channels4(x)).float()
    loss = torch.nn.functional.cross_entropy(out, y)
    loss.backward()
    return out.detach().clone(), {n: p.grad.float().clone() for n, p in m.named_parameters()}


def cmp(tag, a, b):
    o1, g1 = a
    o2, g2 = b
    print(tag, "logits maxdiff", float((o1 - o2).abs().max()), "grad worst rel",
          max(float((g1[n] - g2[n]).abs().max()) / (float(g2[n].abs().max()) + 1e-6) for n in g1), flush=True)


conv.FUSE_BN_BWD = False
for native3 in (False, True):
    resnet.NATIVE_CONV3X3 = native3
    for hw, bs in ((64, 4), (224, 2)):
        cmp(f"native3x3={native3} hw={hw} bs={bs}", run(hw, bs), run(hw, bs))
