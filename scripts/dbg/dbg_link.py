"""Debug: gradient error of fused-BN variants (shortcut link / HIP max-pool) vs stock ResNet-50."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from determined_1_amd.models import resnet  # noqa: E402
from determined_1_amd.ops import norm  # noqa: E402
from determined_1_amd.ops.pool import MaxPool3x3s2  # noqa: E402

gpu = torch.device("cuda", 0)
torch.manual_seed(1)
resnet.FUSED_BN = False
ref = resnet.resnet50(num_classes=10, zero_init_residual=False).to(gpu).to(memory_format=torch.channels_last)
resnet.FUSED_BN = True
base = copy.deepcopy(ref)
for m in base.modules():
    if isinstance(m, norm.BatchNormAct2d):
        m.fused = True
variants = {"base": (base, False, False), "base2": (copy.deepcopy(base), False, False),
            "link": (copy.deepcopy(base), True, False), "pool": (copy.deepcopy(base), False, True),
            "both": (copy.deepcopy(base), True, True), "ref2": (copy.deepcopy(ref), False, False)}
x = torch.randn(8, 3, 64, 64, device=gpu).to(memory_format=torch.channels_last)
t = torch.randint(0, 10, (8,), device=gpu)
sd0 = {k: v.clone() for k, v in ref.state_dict().items()}
torch.nn.functional.cross_entropy(ref(x), t).backward()
for name, (m, link, pool) in variants.items():
    m.load_state_dict(sd0)
    if pool:
        m.maxpool = MaxPool3x3s2()
    norm.SHORTCUT_LINK = link
    torch.nn.functional.cross_entropy(m(x), t).backward()
    errs = {na: ((pb.grad - pa.grad).norm() / pa.grad.norm().clamp_min(1e-12)).item()
            for (na, pa), (_, pb) in zip(ref.named_parameters(), m.named_parameters())}
    top = sorted(errs.items(), key=lambda kv: -kv[1])[:3]
    print(f"{name:6s} max {top[0][1]:.2e} median {sorted(errs.values())[len(errs) // 2]:.2e} "
          f"top {[(k, round(v, 5)) for k, v in top]}", flush=True)
