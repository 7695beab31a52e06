"""Microbenchmark of the MFMA attention kernels (det_attention.hip) at BERT / ALBERT shapes,
with and without probability dropout.  Prints ms per fwd and per fwd+bwd and TFLOP/s."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from determined_1_amd.ops import transformer as tfops  # noqa: E402


def bench(B, S, nh, p, iters=50):
    H = nh * 64
    qkv = torch.randn(B, S, 3 * H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    mb = torch.zeros(B, 1, 1, S, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(B, S, H, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        tfops.qkv_self_attention(qkv, nh, mb, p, training=True).backward(dy)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        with torch.no_grad():
            tfops.qkv_self_attention(qkv, nh, mb, p, training=True)
    torch.cuda.synchronize()
    tf = (time.perf_counter() - t) / iters
    t = time.perf_counter()
    for _ in range(iters):
        tfops.qkv_self_attention(qkv, nh, mb, p, training=True).backward(dy)
    torch.cuda.synchronize()
    tfb = (time.perf_counter() - t) / iters
    flop = 4 * B * nh * S * S * 64
    print(f"B{B} S{S} nh{nh} p={p}: fwd {tf * 1e3:.3f} ms ({flop / tf / 1e12:.0f} TF/s)  "
          f"fwd+bwd {tfb * 1e3:.3f} ms ({3.5 * flop / tfb / 1e12:.0f} TF/s)", flush=True)


if __name__ == "__main__":
    for p in (0.0, 0.1):
        bench(12, 384, 12, p)
    bench(8, 384, 64, 0.0)
