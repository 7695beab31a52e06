"""Microbenchmark of the MFMA attention kernels (det_attention.hip) against torch SDPA (AOTriton /
math on ROCm) at the BERT, ALBERT, DETR and head_dim-128 shapes, with and without probability
dropout.  Prints ms per fwd and per fwd+bwd and TFLOP/s, one JSON line per case; the native
backward both as one merged grid (default) and as two launches.  ``--graph``: GPU time of hipGraph
replays instead of the host loop."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from determined_1_amd.ops import transformer as tfops  # noqa: E402


def _time(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


GRAPH = "--graph" in sys.argv  # time hipGraph replays: GPU time without the autograd host overhead


def _time_graph(fn, iters):
    """fn captured into one hipGraph (after warmup on a side stream) and replayed: the BERT-shape
    fwd+bwd is ~0.1 ms of kernels, which Python autograd dispatch alone can exceed."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters / 1e3


def bench(B, S, nh, hd=64, dt=torch.bfloat16, p=0.0, iters=30, Lk=None):
    Lk = S if Lk is None else Lk
    H = nh * hd
    q, k, v = (torch.randn(B, L, H, device="cuda", dtype=dt, requires_grad=True) for L in (S, Lk, Lk))
    mb = torch.zeros(B, 1, 1, Lk, device="cuda", dtype=dt)
    dy = torch.randn(B, S, H, device="cuda", dtype=dt)

    def native(bwd):
        o = tfops.attention(q, k, v, nh, attn_bias=mb, p=p, training=True)
        if bwd:
            o.backward(dy)

    def heads(t):
        return t.view(B, t.shape[1], nh, hd).transpose(1, 2)

    def sdpa(bwd):
        o = F.scaled_dot_product_attention(heads(q), heads(k), heads(v), attn_mask=mb, dropout_p=p)
        if bwd:
            o.transpose(1, 2).reshape(B, S, H).backward(dy)

    flop = 4 * B * nh * S * Lk * hd
    res = {"B": B, "Lq": S, "Lk": Lk, "nh": nh, "hd": hd, "dtype": str(dt).split(".")[-1], "p": p,
           "timing": "hipgraph replay" if GRAPH else "host loop"}
    from determined_1_amd.ops import _lib

    lib = _lib.get_lib()
    for name, fn in (("native", native), ("native_2launch", native), ("native_merged", native), ("sdpa", sdpa)):
        # native: the default (merged backward grid for small grids); native_2launch: dQ then dK/dV
        # launches; native_merged: always merged
        lib.det_attn_set_bwd_merged({"native": -1, "native_2launch": 0, "native_merged": 1}.get(name, -1))
        if GRAPH:
            if p > 0:
                continue  # dropout RNG state is not graph-safe here
            try:
                with torch.no_grad():
                    tf = _time_graph(lambda: fn(False), iters * 10)
                tfb = _time_graph(lambda: fn(True), iters * 10)
            except Exception as e:  # capture not supported by this path
                res[name] = {"error": f"{type(e).__name__}: {e}"[:200]}
                continue
        else:
            with torch.no_grad():
                tf = _time(lambda: fn(False), iters)
            tfb = _time(lambda: fn(True), iters)
        res[name] = {"fwd_ms": round(tf * 1e3, 4), "fwd_tflops": round(flop / tf / 1e12, 1),
                     "fwd_bwd_ms": round(tfb * 1e3, 4), "fwd_bwd_tflops": round(3.5 * flop / tfb / 1e12, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    for p in (0.0, 0.1):
        bench(12, 384, 12, p=p)  # BERT-base SQuAD
    bench(8, 384, 64, p=0.0)  # ALBERT-xxlarge
    bench(8, 384, 64, dt=torch.float32)  # ALBERT-xxlarge fp32 (reference const.yaml precision)
    bench(2, 850, 8, hd=32, dt=torch.float32)  # DETR encoder fp32
    bench(2, 100, 8, hd=32, dt=torch.float32, Lk=850)  # DETR cross-attention fp32
    bench(4, 1024, 16, hd=128)  # head_dim 128
