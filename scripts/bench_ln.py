"""LayerNorm(dropout(h) + r) forward and backward at the BERT-base shape (4608 x 768 bf16, p = 0.1),
HIP-event time per call and the streaming-bound share of the compulsory bytes.  Kernel variants are
chosen by env (read once per process): DET_LN_FWD=narrow|wide, DET_LN_ROWS=1|2, DET_LN_BWD_BLOCKS.

    python scripts/bench_ln.py [--rows 4608 --hidden 768 --iters 100]
"""
import argparse
import json
import os
import sys
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from determined_1_amd.ops import transformer as tf  # noqa: E402


def timed(fn, iters):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4608)
    ap.add_argument("--hidden", type=int, default=768)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--p", type=float, default=0.1)
    args = ap.parse_args()
    R, H = args.rows, args.hidden
    dev, bf = torch.device("cuda"), torch.bfloat16
    h = torch.randn(R, H, device=dev, dtype=bf)
    r = torch.randn(R, H, device=dev, dtype=bf)
    g = torch.ones(H, device=dev, dtype=bf)
    b = torch.zeros(H, device=dev, dtype=bf)
    dy = torch.randn(R, H, device=dev, dtype=bf)
    y, mean, rstd, seed, off = tf._ln_forward(h, r, g, b, args.p, 1e-12)
    ctx = types.SimpleNamespace(need_gamma=True, need_beta=True, p=args.p, seed=seed, off=off)
    fwd = timed(lambda: tf._ln_forward(h, r, g, b, args.p, 1e-12), args.iters)
    bwd = timed(lambda: tf._ln_backward(ctx, dy, h, r, g, mean, rstd, True, True, True), args.iters)
    mb = R * H * 2 / 1e6
    print(json.dumps({"rows": R, "hidden": H, "env": {k: os.environ.get(k) for k in ("DET_LN_FWD", "DET_LN_ROWS", "DET_LN_BWD_BLOCKS", "DET_LN_BWD")},
                      "fwd_us": round(fwd, 2), "bwd_us": round(bwd, 2),
                      "fwd_TBps": round(3 * mb / fwd, 2), "bwd_TBps_incl_finalize": round(5 * mb / bwd, 2)}))


if __name__ == "__main__":
    main()
