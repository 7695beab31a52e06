"""GEMM host overhead and kernel time for the BERT-base shapes, hipBLASLt vs rocBLAS.

    python scripts/bench_gemm.py
Host overhead = CPU time per launch with the GPU queue kept non-empty (issue rate of tiny GEMMs);
kernel time = HIP-event time per call over 50 back-to-back calls of the real shape.
"""
import json
import time

import torch

SHAPES = {  # (M, K, N) for x[M,K] @ W^T[K,N]; T = 12 * 384 tokens
    "qkv_fwd": (4608, 768, 2304), "out_fwd": (4608, 768, 768), "ffn1_fwd": (4608, 768, 3072),
    "ffn2_fwd": (4608, 3072, 768), "ffn2_dgrad": (4608, 768, 3072), "ffn1_wgrad": (3072, 4608, 768),
}


def run(lib: str) -> dict:
    torch.backends.cuda.preferred_blas_library(lib)
    out = {}
    a = torch.randn(64, 64, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(64, 64, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(64, device="cuda", dtype=torch.bfloat16)
    for _ in range(200):
        torch.addmm(bias, a, b)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(2000):
        torch.addmm(bias, a, b)
    host = (time.perf_counter() - t) / 2000 * 1e6
    torch.cuda.synchronize()
    out["host_us_per_addmm"] = round(host, 2)
    t = time.perf_counter()
    for _ in range(2000):
        a @ b
    out["host_us_per_mm"] = round((time.perf_counter() - t) / 2000 * 1e6, 2)
    torch.cuda.synchronize()
    for name, (M, K, N) in SHAPES.items():
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        bb = torch.randn(N, device="cuda", dtype=torch.bfloat16)
        for _ in range(10):
            torch.addmm(bb, x, w.t())
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            torch.addmm(bb, x, w.t())
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 50
        out[name] = {"us": round(ms * 1e3, 1), "tflops": round(2 * M * K * N / ms / 1e9, 1)}
    return out


if __name__ == "__main__":
    for lib in ("cublaslt", "cublas"):
        print(json.dumps({"lib": lib, **run(lib)}), flush=True)
