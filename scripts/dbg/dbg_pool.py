import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from determined_1_amd.ops import pool

for dt in (torch.float32, torch.bfloat16):
    for (N, C, H, W) in [(1, 8, 6, 6), (1, 16, 8, 8), (2, 64, 112, 112)]:
        torch.manual_seed(0)
        x = torch.randn(N, C, H, W).to(dt).float()
        ref = F.max_pool2d(x, 3, 2, 1)
        out = pool.max_pool_3x3s2(x.to("cuda", dt).contiguous(memory_format=torch.channels_last)).float().cpu()
        bad = (out != ref)
        print(dt, (N, C, H, W), "bad frac", bad.float().mean().item(), flush=True)
        if bad.any():
            idx = bad.nonzero()[:5]
            for i in idx.tolist():
                n, c, oh, ow = i
                print("  at", i, "out", out[n, c, oh, ow].item(), "ref", ref[n, c, oh, ow].item(),
                      "win", x[n, c, max(0, 2*oh-1):2*oh+2, max(0, 2*ow-1):2*ow+2].flatten().tolist())
            # which channels / positions are bad
            print("  bad by channel", bad.float().mean(dim=(0, 2, 3))[:16].tolist())
            print("  bad by oh", bad.float().mean(dim=(0, 1, 3))[:12].tolist())
