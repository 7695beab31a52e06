"""Per-shape timing of ResNet-50's 1x1 convolutions at batch 512 (bf16, NHWC): the hand-written
det_conv GEMMs (forward + fused BN stats, dgrad, wgrad) vs torch/MIOpen conv2d forward and backward.
Prints one JSON line per shape plus totals (x multiplicity in the network).  The forward is timed at
each register prefetch depth of the plain GEMM (det_conv_nt_set_pf 1..3), GEMM-only (no statistics
epilogue) and fused; TF/s and % of the 2.5 PF/s dense bf16 peak are reported for each."""
import json
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from determined_1_amd.ops import _lib, conv  # noqa: E402

PEAK_TF = 2500.0

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
shapes = {}


def add(ci, co, s, h):
    shapes[(ci, co, s, h)] = shapes.get((ci, co, s, h), 0) + 1


inpl = 64
for planes, blocks, stride, h in [(64, 3, 1, 56), (128, 4, 2, 56), (256, 6, 2, 28), (512, 3, 2, 14)]:
    for b in range(blocks):
        s = stride if b == 0 else 1
        hin = h if b == 0 else h // stride
        add(inpl, planes, 1, hin)
        add(planes, planes * 4, 1, hin // s)
        if b == 0:
            add(inpl, planes * 4, s, hin)
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


tot = {"wide_fwd": 0.0, "mine_fwd": 0.0, "mine_fwd_gemm_only": 0.0, "mine_fwd_pf1": 0.0, "mine_dgrad": 0.0, "mine_wgrad": 0.0,
       "miopen_fwd": 0.0, "miopen_bwd": 0.0}
for (ci, co, s, h), mult in shapes.items():
    ho = h // s
    m = N * ho * ho
    x = torch.randn(N, h, h, ci, device=dev).to(torch.bfloat16)
    w = (torch.randn(co, ci, device=dev) / ci ** 0.5).to(torch.bfloat16)
    wt = w.t().contiguous()
    dy = torch.randn(m, co, device=dev).to(torch.bfloat16)
    dw = torch.empty(co, ci, device=dev, dtype=torch.bfloat16)
    g = (ho, ho, h, h) if s == 2 else None
    x2 = x.view(-1, ci)
    fl = 2.0 * m * ci * co
    by_pf = {}
    for pf in (1, 2, 3):
        _lib.get_lib().det_conv_nt_set_pf(pf)
        by_pf[pf] = (timeit(lambda: conv.conv1x1_nt(x2, w, m=m, stats=True, gather=g)),
                     timeit(lambda: conv.conv1x1_nt(x2, w, m=m, stats=False, gather=g)),
                     timeit(lambda: conv.dgrad_1x1(dy, w)) if s == 1 else float("nan"))
    _lib.get_lib().det_conv_nt_set_pf(0)
    # the occupancy-3 128 x 64 tiles of the short-K wide-N forwards (det_conv_nt_set_wide)
    _lib.get_lib().det_conv_nt_set_wide(1)
    wide = (timeit(lambda: conv.conv1x1_nt(x2, w, m=m, stats=True, gather=g)),
            timeit(lambda: conv.conv1x1_nt(x2, w, m=m, stats=False, gather=g)))
    _lib.get_lib().det_conv_nt_set_wide(-1)
    best = min(by_pf, key=lambda p: by_pf[p][0])
    t_f, t_g = by_pf[best][0], by_pf[best][1]
    t_d = min(v[2] for v in by_pf.values()) if s == 1 else float("nan")
    t_w = timeit(lambda: conv.conv1x1_wgrad(dy, x2, dw, gather=g))
    xc = x.permute(0, 3, 1, 2).requires_grad_()  # channels_last NCHW view
    wc = w.view(co, ci, 1, 1).contiguous(memory_format=torch.channels_last).requires_grad_()
    gy = dy.view(N, ho, ho, co).permute(0, 3, 1, 2)
    t_mf = timeit(lambda: F.conv2d(xc, wc, stride=s))
    t_mb = timeit(lambda: torch.autograd.grad(F.conv2d(xc, wc, stride=s), (xc, wc), gy)) - t_mf
    byt_f = (m * ci * (1 if s == 1 else 1) + m * co) * 2
    rec = {"ci": ci, "co": co, "s": s, "h": h, "mult": mult, "M": m,
           "mine_fwd_ms": round(t_f, 4), "mine_fwd_gemm_only_ms": round(t_g, 4), "best_pf": best,
           "fwd_ms_by_pf": {p: round(v[0], 4) for p, v in by_pf.items()},
           "gemm_only_ms_by_pf": {p: round(v[1], 4) for p, v in by_pf.items()},
           "dgrad_bt_ms_by_pf": {p: round(v[2], 4) for p, v in by_pf.items()},
           "wide_fwd_ms": round(wide[0], 4), "wide_gemm_only_ms": round(wide[1], 4),
           "mine_dgrad_ms": round(t_d, 4), "mine_wgrad_ms": round(t_w, 4),
           "miopen_fwd_ms": round(t_mf, 4), "miopen_bwd_ms": round(t_mb, 4),
           "mine_fwd_TBs": round(byt_f / t_f / 1e9, 2), "mine_fwd_TFs": round(fl / t_f / 1e9, 1),
           "gemm_only_TFs": round(fl / t_g / 1e9, 1), "gemm_only_pct_peak": round(100 * fl / t_g / 1e9 / PEAK_TF, 1),
           "miopen_fwd_TFs": round(fl / t_mf / 1e9, 1), "miopen_pct_peak": round(100 * fl / t_mf / 1e9 / PEAK_TF, 1)}
    print(json.dumps(rec), flush=True)
    tot["wide_fwd"] += min(wide[0], t_f) * mult
    tot["mine_fwd"] += t_f * mult
    tot["mine_fwd_gemm_only"] += t_g * mult
    tot["mine_fwd_pf1"] += by_pf[1][0] * mult
    tot["mine_dgrad"] += (t_d if s == 1 else 0.0) * mult
    tot["mine_wgrad"] += t_w * mult
    tot["miopen_fwd"] += t_mf * mult
    tot["miopen_bwd"] += t_mb * mult
print(json.dumps({"totals_ms": {k: round(v, 3) for k, v in tot.items()}}))
