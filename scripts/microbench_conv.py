"""Per-shape timing of ResNet-50 (bs=256, bf16, NHWC) convolutions: MIOpen conv2d vs hipBLASLt GEMM
formulation for 1x1 convs; plus BN/ReLU/add elementwise costs.  Prints one line per shape."""
import sys
import time

import torch
import torch.nn.functional as F

torch.backends.cudnn.benchmark = bool(int(sys.argv[1])) if len(sys.argv) > 1 else False
dev = torch.device("cuda")
N = int(sys.argv[2]) if len(sys.argv) > 2 else 256
# (Cin, Cout, k, stride, H_in) for every distinct conv of ResNet-50 v1.5, with multiplicity
shapes = {}
def add(ci, co, k, s, h):
    shapes[(ci, co, k, s, h)] = shapes.get((ci, co, k, s, h), 0) + 1
add(3, 64, 7, 2, 224)
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
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


tot_conv = tot_mm = 0.0
for (ci, co, k, s, h), mult in shapes.items():
    x = torch.randn(N, ci, h, h, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_()
    w = torch.randn(co, ci, k, k, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_()
    y = F.conv2d(x, w, stride=s, padding=k // 2)
    gy = torch.randn_like(y)

    def conv_fb():
        out = F.conv2d(x, w, stride=s, padding=k // 2)
        out.backward(gy)
    t_conv = timeit(conv_fb)
    flops = 2 * N * y.shape[2] * y.shape[3] * co * ci * k * k * 3
    line = f"conv ci={ci:4d} co={co:4d} k={k} s={s} h={h:3d} x{mult}: miopen fwd+bwd {t_conv:7.3f} ms ({flops / t_conv / 1e9:6.1f} TF)"
    tot_conv += t_conv * mult
    if k == 1 and s == 1:
        xm = x.detach().permute(0, 2, 3, 1).reshape(-1, ci).requires_grad_()
        wm = w.detach().reshape(co, ci).requires_grad_()
        gym = gy.permute(0, 2, 3, 1).reshape(-1, co)

        def mm_fb():
            out = xm @ wm.t()
            out.backward(gym)
        t_mm = timeit(mm_fb)
        line += f" | gemm {t_mm:7.3f} ms ({flops / t_mm / 1e9:6.1f} TF)"
        tot_mm += min(t_mm, t_conv) * mult
    else:
        tot_mm += t_conv * mult
    print(line, flush=True)
print(f"TOTAL conv fwd+bwd per step: miopen {tot_conv:.2f} ms, best-of(miopen,gemm for 1x1) {tot_mm:.2f} ms")

# BN + ReLU costs at the biggest activation (N,256,56,56)
for c, h in [(64, 112), (256, 56), (512, 28), (1024, 14)]:
    x = torch.randn(N, c, h, h, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_()
    bn = torch.nn.BatchNorm2d(c).to(dev).to(memory_format=torch.channels_last)
    gy = torch.randn_like(x)

    def bn_fb():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = torch.relu(bn(x))
        out.backward(gy)
    t = timeit(bn_fb)
    gb = x.numel() * 2 / 1e9
    print(f"bn+relu fwd+bwd c={c} h={h}: {t:.3f} ms  ({gb:.2f} GB activation; {11 * gb / t:.0f} GB/s at 11 passes)")
