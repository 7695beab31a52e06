"""ResNet-50 stem (7x7/2 conv, 64 filters, 224x224 input, batch 512) on MIOpen: forward and weight
gradient time with the input channels padded from 3 to 4 or 8 (zero channels, zero weights --
the same convolution), channels_last bf16.  Prints one JSON line per variant."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main() -> None:
    torch.backends.cudnn.benchmark = True
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    x3 = torch.randn(n, 3, 224, 224, generator=g).to(dev, torch.bfloat16)
    w3 = (torch.randn(64, 3, 7, 7, generator=g) * 0.1).to(dev, torch.bfloat16)
    ref = None
    for c in (3, 4, 8):
        x = torch.zeros(n, c, 224, 224, device=dev, dtype=torch.bfloat16)
        x[:, :3] = x3
        x = x.contiguous(memory_format=torch.channels_last)
        w = torch.zeros(64, c, 7, 7, device=dev, dtype=torch.bfloat16)
        w[:, :3] = w3
        w = w.contiguous(memory_format=torch.channels_last)
        y = F.conv2d(x, w, stride=2, padding=3)
        dy = torch.randn_like(y)
        fwd = timeit(lambda: F.conv2d(x, w, stride=2, padding=3))
        wgrad = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1, [False, True, False]))
        err = None
        if ref is None:
            ref = y.float()
        else:
            err = float((y.float() - ref).abs().max())
        print(json.dumps({"impl": "miopen", "cin": c, "batch": n, "fwd_ms": round(fwd, 4), "wgrad_ms": round(wgrad, 4),
                          "max_abs_diff_vs_c3": err}), flush=True)
        if c == 4:
            from determined_1_amd.ops import conv as nc

            cv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(dev)
            with torch.no_grad():
                cv.weight.copy_(w3.float())
            cv = cv.to(torch.bfloat16)
            cvp = cv.weight.detach().requires_grad_(True)
            fwd_n = timeit(lambda: nc._StemConv.apply(x, cvp, True))
            yn = nc._StemConv.apply(x, cvp, True)
            nc.STEM_NATIVE_WGRAD = True
            wgrad_n = timeit(lambda: torch.autograd.grad(yn, cvp, dy, retain_graph=True))
            print(json.dumps({"impl": "det_conv GM_STEM (+BN stats; native split-M wgrad)",
                              "cin": 4, "batch": n, "fwd_ms": round(fwd_n, 4), "wgrad_ms": round(wgrad_n, 4),
                              "max_abs_diff_vs_miopen": float((yn.float() - ref).abs().max())}), flush=True)


if __name__ == "__main__":
    main()
