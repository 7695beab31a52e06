"""Time det_gemm8 (both staging schedules) against torch.mm (hipBLASLt) on the BERT-base Linear
shapes and a few square sizes: median of CUDA-event timings, TF/s.
    python scripts/bench_gemm8.py [--iters 50]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from determined_1_amd.ops.gemm8 import gemm8  # noqa: E402

SHAPES = {  # name: (M, N, K) for C = A . B^T
    "qkv_fwd": (4608, 2304, 768), "ffn_in_fwd": (4608, 3072, 768), "ffn_out_fwd": (4608, 768, 3072),
    "attn_out_fwd": (4608, 768, 768), "qkv_dgrad": (4608, 768, 2304), "ffn_in_dgrad": (4608, 768, 3072),
    "ffn_out_dgrad": (4608, 3072, 768), "qkv_wgrad": (2304, 768, 4608), "ffn_in_wgrad": (3072, 768, 4608),
    "ffn_out_wgrad": (768, 3072, 4608), "sq4096": (4096, 4096, 4096), "sq8192": (8192, 8192, 8192),
    # ResNet-50 3x3 convolutions as dense GEMMs (pixels x Cout x 9*Cin) at 512 images
    "conv3x3_c256": (100352, 256, 2304), "conv3x3_c512": (25088, 512, 4608),
}


def timeit(fn, iters, reps=20):
    """Median over `iters` samples of the per-launch time of `reps` back-to-back launches (the
    launch latency is hidden as it is inside a step)."""
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / reps)
    ts.sort()
    return ts[len(ts) // 2] * 1e3  # us


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=15)
    ap.add_argument("--only", default="")
    ap.add_argument("--modes", default="0,1", help="det_gemm8 schedule variants (det_gemm8.hip MODE bits)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    for name, (m, n, k) in SHAPES.items():
        if args.only and name not in args.only.split(","):
            continue
        a = torch.rand(m, k, device=dev).sub(0.5).to(torch.bfloat16)
        b = torch.rand(n, k, device=dev).sub(0.5).to(torch.bfloat16)
        out = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        flop = 2.0 * m * n * k
        rec = {"shape": name, "M": m, "N": n, "K": k}
        rec["blas_us"] = round(timeit(lambda: torch.mm(a, b.t(), out=out), args.iters), 2)
        for mode in [int(x) for x in args.modes.split(",")]:
            rec[f"gemm8_m{mode}_us"] = round(timeit(lambda: gemm8(a, b, out=out, mode=mode), args.iters), 2)
        for key in [k_ for k_ in rec if k_.endswith("_us")]:
            rec[key.replace("_us", "_tfs")] = round(flop / rec[key] / 1e6, 1)
        ref = (a.float() @ b.float().t())
        rec["max_rel_err"] = float((gemm8(a, b).float() - ref).abs().max() / ref.abs().max())
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
