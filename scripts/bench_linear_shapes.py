"""BERT-base Linear GEMMs (12 x 384 tokens): the vendor BLAS through torch (with the shipped tuned
solutions, ops/gemm_tuning.py) against the hand-written det_conv.hip tiles (DET_NATIVE_LINEAR),
per pass, in TF/s of HIP-event time over back-to-back calls.

    python scripts/bench_linear_shapes.py [--iters 30]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from determined_1_amd.ops import _lib, gemm_tuning
from determined_1_amd.ops.conv import conv1x1_wgrad, dgrad_1x1

T = 4608
LAYERS = {"qkv": (768, 2304), "attn_out": (768, 768), "ffn_in": (768, 3072), "ffn_out": (3072, 768)}  # (K in, N out)


def timed(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--igemm", default="", help="comma-separated det_igemm tile cfgs to time as plain GEMMs")
    ap.add_argument("--wgcfg", default="", help="comma-separated det_igemm_wgrad cfgs (1x1 geometry)")
    args = ap.parse_args()
    tuned = gemm_tuning.enable()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    res = {"tuned_file_loaded": tuned, "tokens": T, "passes": {}}
    lib = _lib.get_lib()
    for name, (K, N) in LAYERS.items():
        x = torch.randn(T, K, device=dev, dtype=bf)
        w = torch.randn(N, K, device=dev, dtype=bf) * 0.02
        b = torch.zeros(N, device=dev, dtype=bf)
        dz = torch.randn(T, N, device=dev, dtype=bf)
        wg = torch.empty(N, K, device=dev, dtype=bf)
        y = torch.empty(T, N, device=dev, dtype=bf)
        st = torch.cuda.current_stream().cuda_stream
        flops = 2.0 * T * K * N
        cases = {
            "fwd/blas": lambda: torch.addmm(b, x, w.t()),
            "fwd/native": lambda: lib.det_linear_fwd(st, x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), T, N, K),
            "dgrad/blas": lambda: dz @ w,
            "dgrad/native": lambda: dgrad_1x1(dz, w),
            "wgrad/blas": lambda: torch.mm(dz.t(), x, out=wg),
            "wgrad/native": lambda: conv1x1_wgrad(dz, x, wg),
        }
        zero = torch.zeros(64, device=dev, dtype=bf)
        wt = w.t().contiguous()  # [K, N]: the input gradient's B operand as the NT kernel reads it
        dx = torch.empty(T, K, device=dev, dtype=bf)

        def ig(cfg, X, W, Y, M, Nn, Kk):
            # X [M, Kk] as a 1 x M image of Kk channels, W [Nn, Kk]: Y = X W^T
            return lambda: _lib.check(lib.det_igemm_conv_cfg(st, X.data_ptr(), W.data_ptr(), Y.data_ptr(), zero.data_ptr(),
                                                             M, Nn, Kk, 1, M, 1, M, 1, 1, 1, 0, None, None, cfg), "ig")

        for c in [int(v) for v in args.igemm.split(",") if v]:
            cases[f"fwd/igemm{c}"] = ig(c, x, w, y, T, N, K)
            cases[f"dgrad/igemm{c}"] = ig(c, dz, wt, dx, T, K, N)
        for c in [int(v) for v in args.wgcfg.split(",") if v]:
            n_ws = int(lib.det_igemm_wgrad_ws_elems(T, N, K, c))
            if n_ws <= 0:
                continue
            ws = torch.empty(n_ws, device=dev, dtype=torch.float32)
            cases[f"wgrad/wg{c}"] = (lambda ws=ws, c=c: _lib.check(lib.det_igemm_wgrad(
                st, dz.data_ptr(), x.data_ptr(), wg.data_ptr(), 1, T, N, K, 1, T, 1, T, 1, 1, 1, 0, ws.data_ptr(),
                1.0, c), "wg"))
        for cname, fn in cases.items():
            try:
                us = timed(fn, args.iters)
            except RuntimeError as e:  # a tile that does not fit the shape
                res["passes"][f"{name}/{cname}"] = {"error": str(e)[:80]}
                continue
            res["passes"][f"{name}/{cname}"] = {"us": round(us, 2), "tflops": round(flops / us / 1e6, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
