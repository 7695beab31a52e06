"""Which parts of a train step survive hipGraph capture on this ROCm/PyTorch build.
    python scripts/dbg/graph_probe.py {mlp|conv_native|conv_miopen} [--no-opt]"""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
case = sys.argv[1]
use_opt = "--no-opt" not in sys.argv
if "--bench" in sys.argv:
    torch.backends.cudnn.benchmark = True
if case == "conv_native":
    torch.backends.cudnn.enabled = False
torch.manual_seed(0)
dev = torch.device("cuda", 0)
if case == "mlp":
    net = nn.Sequential(nn.Flatten(), nn.Linear(3 * 16 * 16, 64), nn.ReLU(), nn.Linear(64, 10)).to(dev)
elif "--maxpool" in sys.argv:
    net = nn.Sequential(nn.Conv2d(3, 16, 3, padding=1), nn.ReLU(), nn.MaxPool2d(2), nn.Conv2d(16, 32, 3, padding=1),
                        nn.ReLU(), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(32, 10)).to(dev)
else:
    net = nn.Sequential(nn.Conv2d(3, 16, 3, padding=1), nn.ReLU(), nn.Conv2d(16, 32, 3, padding=1), nn.ReLU(),
                        nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(32, 10)).to(dev)
opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
if use_opt:
    from determined_1_amd.ops.optim import FusedOptimizer

    FusedOptimizer(opt, dev)
x = torch.randn(16, 3, 16, 16, device=dev)
y = torch.randint(0, 10, (16,), device=dev)


def step():
    out = net(x)
    loss = nn.functional.cross_entropy(out, y)
    loss.backward()
    opt.step()
    opt.zero_grad()
    return loss


for _ in range(3):
    step()
torch.cuda.synchronize()
print(case, "eager ok", flush=True)
g = torch.cuda.CUDAGraph()
xs = x.clone()
x = xs
with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle()):
    loss = step()
print(case, "captured", flush=True)
for _ in range(5):
    g.replay()
torch.cuda.synchronize()
print(case, "replay ok loss", float(loss), flush=True)
