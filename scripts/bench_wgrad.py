"""ResNet-50 (batch 512, bf16, NHWC) weight-gradient timing for every conv shape of the network:
det_igemm_wgrad (LDS-DMA ring + transposed reads) per tile configuration vs det_conv's gemm_tn vs
MIOpen (torch.ops.aten.convolution_backward weight only).  One JSON line per (shape, candidate),
then weighted totals per candidate and for the per-shape best ring configuration.

    python scripts/bench_wgrad.py [--batch 512] [--cfgs 1,...,9]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from determined_1_amd.ops import conv  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--batch", type=int, default=512)
p.add_argument("--cfgs", default="1,2,3,4,5,6,7,8,9,10,11,12,13")
p.add_argument("--iters", type=int, default=20)
p.add_argument("--only-r", type=int, default=0, help="restrict to 1x1 (1) or 3x3 (3) shapes")
args = p.parse_args()
torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
NB = args.batch

shapes = {}  # (cin, cout, r, stride, hin) -> count
inpl = 64
for planes, blocks, stride, h in [(64, 3, 1, 56), (128, 4, 2, 56), (256, 6, 2, 28), (512, 3, 2, 14)]:
    for b in range(blocks):
        s = stride if b == 0 else 1
        hin = h if b == 0 else h // stride
        ks = [(inpl, planes, 1, 1, hin), (planes, planes, 3, s, hin), (planes, planes * 4, 1, 1, hin // s)]
        if b == 0:
            ks.append((inpl, planes * 4, 1, s, hin))
        for k in ks:
            shapes[k] = shapes.get(k, 0) + 1
        inpl = planes * 4


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / args.iters


tot = {}
best_tot = 0.0
for (cin, cout, r, st, hin), mult in shapes.items():
    if args.only_r and r != args.only_r:
        continue
    pad = r // 2
    ho = (hin + 2 * pad - r) // st + 1
    m = NB * ho * ho
    x = torch.randn(NB, cin, hin, hin, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(cout, cin, r, r, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(NB, cout, ho, ho, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out = torch.empty(cout, r * r * cin, dtype=torch.bfloat16, device=dev)
    flops = 2.0 * m * cout * cin * r * r
    base = {"cin": cin, "cout": cout, "r": r, "stride": st, "hin": hin, "mult": mult, "M": m}
    ref = torch.ops.aten.convolution_backward(dy, x, w, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
                                              [False, True, False])[1].float()
    res = {}
    res["miopen"] = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [st, st], [pad, pad], [1, 1], False,
                                                                       [0, 0], 1, [False, True, False]))
    if cin % 64 == 0:
        res["gemm_tn"] = timeit(lambda: conv.conv_wgrad(dy, x, out, r, r, st, pad, cfg=-1))
    best = None
    for cfg in [int(c) for c in args.cfgs.split(",") if c]:
        try:
            conv.conv_wgrad(dy, x, out, r, r, st, pad, cfg=cfg)
        except RuntimeError:
            continue
        got = out.view(cout, r, r, cin).permute(0, 3, 1, 2).float()
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        ms = timeit(lambda: conv.conv_wgrad(dy, x, out, r, r, st, pad, cfg=cfg))
        res["ring%d" % cfg] = ms
        print(json.dumps(dict(base, cand="ring%d" % cfg, ms=round(ms, 4), TFs=round(flops / ms / 1e9, 1),
                              rel_err=round(err, 5))), flush=True)
        if best is None or ms < res[best]:
            best = "ring%d" % cfg
    for k in ("miopen", "gemm_tn"):
        if k in res:
            print(json.dumps(dict(base, cand=k, ms=round(res[k], 4), TFs=round(flops / res[k] / 1e9, 1))), flush=True)
    for k, v in res.items():
        tot[k] = tot.get(k, 0.0) + v * mult
    if best:
        best_tot += res[best] * mult
        print(json.dumps(dict(base, best=best, best_ms=round(res[best], 4), miopen_ms=round(res["miopen"], 4))), flush=True)
print(json.dumps({"totals_ms": {k: round(v, 3) for k, v in sorted(tot.items(), key=lambda kv: kv[1])},
                  "best_ring_total_ms": round(best_tot, 3)}))
