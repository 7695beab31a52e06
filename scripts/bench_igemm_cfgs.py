"""det_igemm tile-configuration sweep over ResNet-50's (batch 512, bf16, NHWC) 1x1 convolutions:
forward (X[M, Cin] x W[Cout, Cin]^T, stats epilogue on) and input gradient (dY[M, Cout] x W as the
same GEMM with the roles swapped), against the register-staged det_conv GEMM (gemm_nt, what the
ResNet path runs) and MIOpen.  One JSON line per (shape, direction, candidate).

    python scripts/bench_igemm_cfgs.py [--batch 512] [--cfgs 2,8,9,11,12,13]
"""
import argparse
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from determined_1_amd.ops import conv  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--batch", type=int, default=512)
p.add_argument("--cfgs", default="2,3,8,9,11,12,13")
p.add_argument("--iters", type=int, default=20)
args = p.parse_args()
torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
NB = args.batch
CFGS = [int(c) for c in args.cfgs.split(",") if c]

shapes = {}  # (cin, cout, stride, hin) -> count
inpl = 64
for planes, blocks, stride, h in [(64, 3, 1, 56), (128, 4, 2, 56), (256, 6, 2, 28), (512, 3, 2, 14)]:
    for b in range(blocks):
        s = stride if b == 0 else 1
        hin = h if b == 0 else h // stride
        for k in [(inpl, planes, 1, hin), (planes, planes * 4, 1, hin // s)] + ([(inpl, planes * 4, s, hin)] if b == 0 else []):
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


def emit(rec, key, ms, mult):
    rec = dict(rec, cand=key, ms=round(ms, 4))
    print(json.dumps(rec), flush=True)
    tot.setdefault(rec["dir"], {}).setdefault(key, 0.0)
    tot[rec["dir"]][key] += ms * mult


for (cin, cout, st, hin), mult in shapes.items():
    ho = (hin - 1) // st + 1
    m = NB * ho * ho
    x = torch.randn(NB, cin, hin, hin, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 1, 1, device=dev) / cin ** 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wk = conv.krsc(w)
    ref = F.conv2d(x, w, stride=st).float()
    flops = 2.0 * m * cout * cin
    byts = 2.0 * (NB * hin * hin * cin + m * cout + cin * cout)
    base = {"cin": cin, "cout": cout, "stride": st, "hin": hin, "mult": mult, "M": m, "dir": "fwd"}
    emit(base, "miopen", timeit(lambda: F.conv2d(x, w, stride=st)), mult)
    if st == 1:
        x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
        emit(base, "det_conv_stats", timeit(lambda: conv.conv1x1_nt(x2, wk, stats=True)), mult)
    for cfg in CFGS:
        try:
            y, _ = conv.igemm_conv(x, w, stride=st, stats=True, w_krsc=wk, cfg=cfg)
        except RuntimeError as e:  # unsupported tile for this shape
            continue
        err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
        ms = timeit(lambda: conv.igemm_conv(x, w, stride=st, stats=True, w_krsc=wk, cfg=cfg))
        r = dict(base, rel_err=round(err, 5), TFs=round(flops / ms / 1e9, 1), TBs=round(byts / ms / 1e9, 2))
        emit(r, "igemm%d" % cfg, ms, mult)
    if st != 1:
        continue
    # input gradient: dX[M, Cin] = dY[M, Cout] x W[Cout, Cin] -> igemm with X := dY, W := W^T
    dy = torch.randn(NB, cout, ho, ho, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = w.reshape(cout, cin).t().contiguous()
    wt4 = wt.view(cin, cout, 1, 1)
    refd = F.conv2d(dy, wt4.contiguous(memory_format=torch.channels_last)).float()
    based = dict(base, dir="dgrad")
    dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
    emit(based, "det_conv", timeit(lambda: conv.conv1x1_nt(dy2, wt)), mult)
    for cfg in CFGS:
        try:
            y, _ = conv.igemm_conv(dy, wt4, stride=1, w_krsc=wt, cfg=cfg)
        except RuntimeError:
            continue
        err = ((y.float() - refd).abs().max() / refd.abs().max()).item()
        ms = timeit(lambda: conv.igemm_conv(dy, wt4, stride=1, w_krsc=wt, cfg=cfg))
        emit(dict(based, rel_err=round(err, 5), TFs=round(flops / ms / 1e9, 1)), "igemm%d" % cfg, ms, mult)
print(json.dumps({"totals_ms": {d: {k: round(v, 3) for k, v in sorted(t.items(), key=lambda kv: kv[1])} for d, t in tot.items()}}))
