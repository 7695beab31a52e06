"""ResNet-50 projection shortcuts (1x1, stride 1 / 2) at batch 512, bf16 NHWC: the native path
(ops.conv._Shortcut1x1 pieces: det_igemm / gemm_nt forward with BN statistics, 1x1 dgrad on the
output grid, gathered gemm_tn or ring weight gradient) against MIOpen's conv2d forward and backward.
One JSON line per shape."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from determined_1_amd.ops import conv  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 512


def timeit(fn, iters=20):
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


for ci, co, s, h in [(64, 256, 1, 56), (256, 512, 2, 56), (512, 1024, 2, 28), (1024, 2048, 2, 14)]:
    ho = h // s
    m = N * ho * ho
    x = torch.randn(N, ci, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(co, ci, 1, 1, device=dev) / ci ** 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wk = w.reshape(co, ci).contiguous()
    dy = torch.randn(N, co, ho, ho, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy2 = dy.permute(0, 2, 3, 1).reshape(-1, co)
    x2 = x.permute(0, 2, 3, 1).reshape(-1, ci)
    dw = torch.empty(co, ci, device=dev, dtype=torch.bfloat16)
    g = (ho, ho, h, h) if s == 2 else None
    rec = {"ci": ci, "co": co, "s": s, "h": h, "M": m}
    if s == 2:
        rec["fwd_igemm8"] = timeit(lambda: conv.igemm_conv(x, w, stride=2, stats=True, w_krsc=wk, cfg=8))
    elif (ci, co) in conv.IGEMM_FWD_1X1:
        rec["fwd_igemm"] = timeit(lambda: conv.igemm_conv(x, w, stats=True, w_krsc=wk, cfg=conv.IGEMM_FWD_1X1[(ci, co)]))
    rec["fwd_gemm_nt"] = timeit(lambda: conv.conv1x1_nt(x2, wk, m=m, stats=True, gather=g))
    rec["dgrad"] = timeit(lambda: conv.dgrad_1x1(dy2, wk))
    rec["wgrad_tn"] = timeit(lambda: conv.conv1x1_wgrad(dy2, x2, dw, gather=g))
    old = conv.WGRAD_RING
    conv.WGRAD_RING = True
    if int(conv._lib.get_lib().det_igemm_wgrad_ws_elems(m, co, ci, 0)) > 0:
        rec["wgrad_ring"] = timeit(lambda: conv.conv_wgrad(dy, x, dw.view(co, ci), 1, 1, s, 0))
    conv.WGRAD_RING = old
    xc = x.clone().requires_grad_()
    wc = w.clone().requires_grad_()
    rec["miopen_fwd"] = timeit(lambda: F.conv2d(xc, wc, stride=s))
    rec["miopen_bwd"] = timeit(lambda: torch.autograd.grad(F.conv2d(xc, wc, stride=s), (xc, wc), dy)) - rec["miopen_fwd"]
    # numerics of the native pieces against fp32
    ref = F.conv2d(x.float(), w.float(), stride=s)
    y, _ = (conv.igemm_conv(x, w, stride=2, stats=True, w_krsc=wk, cfg=8) if s == 2 else
            (conv.conv1x1_nt(x2, wk, stats=True)[0].view(N, ho, ho, co).permute(0, 3, 1, 2), None))
    rec["fwd_rel_err"] = float((y.float() - ref).abs().max() / ref.abs().max())
    gw = torch.nn.grad.conv2d_weight(x.float(), (co, ci, 1, 1), dy.float(), stride=s).view(co, ci)
    conv.conv1x1_wgrad(dy2, x2, dw, gather=g)
    rec["wgrad_rel_err"] = float((dw.float() - gw).abs().max() / gw.abs().max())
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in rec.items()}), flush=True)
