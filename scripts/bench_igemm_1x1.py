"""ResNet-50's 1x1 convolutions (batch 512, bf16 NHWC) on det_igemm with the BN-statistics epilogue:
the automatic tile configuration vs the eight-phase cfg 21 (256 x 256) / 22 (512 x 128) where they
fit.  One JSON line per shape (ms per call).   python scripts/bench_igemm_1x1.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from determined_1_amd.ops import conv  # noqa: E402

NB = 512
SHAPES = [(64, 256, 56, 1), (128, 512, 28, 1), (256, 1024, 14, 1), (512, 2048, 7, 1), (1024, 256, 14, 1),
          (2048, 512, 7, 1), (256, 512, 56, 2), (512, 1024, 28, 2), (1024, 2048, 14, 2), (512, 128, 28, 1)]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(3):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / iters)
    return sorted(ts)[1]


dev = torch.device("cuda")
CFGS = [int(c) for c in os.environ.get("CFGS", "0,8,21,22").split(",")]
STATS = os.environ.get("STATS", "1") == "1"
for cin, cout, h, st in SHAPES:
    x = torch.randn(NB, cin, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 1, 1, device=dev) / cin ** 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    r = {"cin": cin, "cout": cout, "h": h, "stride": st}
    r["stats"] = STATS
    for cfg in CFGS:
        try:
            r[f"cfg{cfg}_ms"] = round(timeit(lambda: conv.igemm_conv(x, w, stride=st, pad=0, stats=STATS, cfg=cfg)), 4)
        except RuntimeError as e:
            r[f"cfg{cfg}_ms"] = None
    print(json.dumps(r), flush=True)
