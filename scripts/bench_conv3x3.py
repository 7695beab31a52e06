"""ResNet-50 (batch 512, bf16, NHWC) 3x3-conv pass timing, native vs MIOpen, in one process:
forward (det_igemm auto cfg, with the BN-statistics epilogue) vs F.conv2d; input gradient (stride
1: det_igemm on the flipped weight incl. the flip kernel) vs MIOpen; weight gradient (det_conv
im2col split-M GEMM) vs MIOpen.  One JSON line per conv shape (with its multiplicity), then totals.

    python scripts/bench_conv3x3.py [batch]
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
SHAPES = [(64, 1, 56, 3), (128, 2, 56, 1), (128, 1, 28, 3), (256, 2, 28, 1), (256, 1, 14, 5), (512, 2, 14, 1),
          (512, 1, 7, 2)]  # (channels, stride, input H, count in ResNet-50)


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(3):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) / iters)
    return sorted(best)[1]


tot = {}
for c, st, hin, mult in SHAPES:
    x = torch.randn(NB, c, hin, hin, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(c, c, 3, 3, device=dev) / (9 * c) ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ho = (hin - 1) // st + 1
    dy = torch.randn(NB, c, ho, ho, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    flops = 2.0 * NB * ho * ho * c * c * 9
    wk = conv.krsc(w)
    r = {"c": c, "stride": st, "hin": hin, "mult": mult}
    r["fwd_native"] = timeit(lambda: conv.igemm_conv(x, w, stride=st, pad=1, stats=True, w_krsc=wk))
    if conv.conv3p_ok(c, c, 3, 3, st, 1):  # the igemm3 path it replaces, for the record
        keep, conv.CONV3P_MAX_N = conv.CONV3P_MAX_N, 0
        r["fwd_igemm3"] = timeit(lambda: conv.igemm_conv(x, w, stride=st, pad=1, stats=True, w_krsc=wk))
        r["dgrad_igemm3"] = timeit(lambda: conv.igemm_conv(dy, w.transpose(0, 1), stride=1, pad=1,
                                                           w_krsc=conv.dgrad_weight(w)))
        conv.CONV3P_MAX_N = keep
    r["fwd_miopen"] = timeit(lambda: F.conv2d(x, w, stride=st, padding=1))
    if st == 1:
        r["dgrad_native"] = timeit(lambda: conv.igemm_conv(dy, w.transpose(0, 1), stride=1, pad=1,
                                                           w_krsc=conv.dgrad_weight(w)))
    else:  # parity-class implicit GEMMs (incl. the flip kernel)
        r["dgrad_native"] = timeit(lambda: conv.igemm_dgrad_s2(dy, w, hin, hin))
    r["dgrad_miopen"] = timeit(lambda: torch.ops.aten.convolution_backward(
        dy, x, w, None, [st, st], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]))
    out = torch.empty(c, 9 * c, dtype=torch.bfloat16, device=dev)
    r["wgrad_native"] = timeit(lambda: conv.conv_wgrad(dy, x, out, 3, 3, st, 1))
    if conv.conv3p_wgrad_ok(c, c, 3, 3, st, 1):  # halo-patch wgrad (the model's choice at these shapes)
        r["wgrad_conv3p"] = timeit(lambda: conv.conv3p_wgrad(dy, x, out))
    r["wgrad_miopen"] = timeit(lambda: torch.ops.aten.convolution_backward(
        dy, x, w, None, [st, st], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
    for k in list(r):
        if k.endswith("_native") or k.endswith("_miopen") or k.endswith("_igemm3") or k.endswith("_conv3p"):
            tot[k] = tot.get(k, 0.0) + mult * r[k]
            r[k.replace("native", "TFs_native").replace("miopen", "TFs_miopen") if False else k] = round(r[k], 4)
            r[k + "_TFs"] = round(flops / r[k] / 1e9, 1)
    print(json.dumps(r), flush=True)
print(json.dumps({"totals_ms_per_step": {k: round(v, 3) for k, v in sorted(tot.items())}}), flush=True)
