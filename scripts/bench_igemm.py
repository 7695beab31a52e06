"""ResNet-50 (batch 512, bf16, NHWC) forward-conv timing: det_igemm (pipelined implicit GEMM) vs
torch/MIOpen conv2d vs the register-staged det_conv 1x1 GEMM.  One JSON line per conv shape with
its multiplicity in the network, then totals.

    python scripts/bench_igemm.py [batch]
"""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from determined_1_amd.ops import conv  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
NB = int(sys.argv[1]) if len(sys.argv) > 1 else 512

shapes = {}  # (cin, cout, r, stride, hin) -> count


def add(*k):
    shapes[k] = shapes.get(k, 0) + 1


inpl = 64
for planes, blocks, stride, h in [(64, 3, 1, 56), (128, 4, 2, 56), (256, 6, 2, 28), (512, 3, 2, 14)]:
    for b in range(blocks):
        s = stride if b == 0 else 1
        hin = h if b == 0 else h // stride
        add(inpl, planes, 1, 1, hin)
        add(planes, planes, 3, s, hin)
        add(planes, planes * 4, 1, 1, hin // s)
        if b == 0:
            add(inpl, planes * 4, 1, s, hin)
        inpl = planes * 4


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


tot = {"igemm": 0.0, "igemm_stats": 0.0, "miopen": 0.0, "det_conv": 0.0}
for (cin, cout, r, st, hin), mult in shapes.items():
    pad = r // 2
    x = torch.randn(NB, cin, hin, hin, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, r, r, device=dev) / (cin * r * r) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    wk = conv.krsc(w)
    ho = (hin + 2 * pad - r) // st + 1
    m = NB * ho * ho
    t_ig = timeit(lambda: conv.igemm_conv(x, w, stride=st, pad=pad, w_krsc=wk))
    t_igs = timeit(lambda: conv.igemm_conv(x, w, stride=st, pad=pad, stats=True, w_krsc=wk))
    t_mi = timeit(lambda: F.conv2d(x, w, stride=st, padding=pad))
    t_dc = float("nan")
    if r == 1:
        x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
        g = None if st == 1 else (ho, ho, hin, hin)
        t_dc = timeit(lambda: conv.conv1x1_nt(x2, wk, m=m, gather=g, stats=True))
    # correctness spot check against MIOpen
    y, _ = conv.igemm_conv(x, w, stride=st, pad=pad, w_krsc=wk)
    err = (y.float() - F.conv2d(x, w, stride=st, padding=pad).float()).abs().max().item()
    flops = 2.0 * m * cout * cin * r * r
    rec = {"cin": cin, "cout": cout, "r": r, "stride": st, "hin": hin, "mult": mult, "M": m,
           "igemm_ms": round(t_ig, 4), "igemm_stats_ms": round(t_igs, 4), "miopen_ms": round(t_mi, 4),
           "det_conv_ms": round(t_dc, 4), "igemm_TFs": round(flops / t_ig / 1e9, 1),
           "miopen_TFs": round(flops / t_mi / 1e9, 1), "max_abs_err_vs_miopen": err}
    print(json.dumps(rec), flush=True)
    tot["igemm"] += mult * t_ig
    tot["igemm_stats"] += mult * t_igs
    tot["miopen"] += mult * t_mi
    if r == 1:
        tot["det_conv"] += mult * t_dc
print(json.dumps({"totals_fwd_ms": {k: round(v, 3) for k, v in tot.items()}}))
