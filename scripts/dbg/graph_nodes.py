"""What does a captured library op put into a hipGraph?  (Round-6 follow-up to the r5 MIOpen replay
divergence: conv1_bwd_weight -- bf16, Cin = 3 -- is the one op whose K-call graph diverges from eager
once eager MIOpen calls run between replays, profiles/r5_graph_nan_root_cause.txt.)

For each op it captures one call with keep_graph=True and lists the graph's nodes: kernels, memsets,
and memcpy nodes with their direction and whether the source is pageable host memory.  A memcpy node
that reads pageable host memory re-reads that host buffer AT REPLAY TIME: if the library rewrites the
buffer on its next (eager) call -- e.g. a kernel-argument block holding tensor pointers -- the replay
uses the eager call's values.

    python scripts/dbg/graph_nodes.py [--dtype bf16]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from miopen_graph_repro import cases  # noqa: E402

NODE_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty", 6: "wait_event",
              7: "event_record", 10: "mem_alloc", 11: "mem_free", 12: "memcpy_from_symbol", 13: "memcpy_to_symbol"}


class _Pos(ctypes.Structure):
    _fields_ = [("x", ctypes.c_size_t), ("y", ctypes.c_size_t), ("z", ctypes.c_size_t)]


class _Pitched(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("pitch", ctypes.c_size_t), ("xsize", ctypes.c_size_t),
                ("ysize", ctypes.c_size_t)]


class _Memcpy3D(ctypes.Structure):
    _fields_ = [("srcArray", ctypes.c_void_p), ("srcPos", _Pos), ("srcPtr", _Pitched), ("dstArray", ctypes.c_void_p),
                ("dstPos", _Pos), ("dstPtr", _Pitched), ("extent", _Pos), ("kind", ctypes.c_int)]


class _PtrAttr(ctypes.Structure):  # hipPointerAttribute_t (type first)
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def _hip():
    for name in ("libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"):
        try:
            return ctypes.CDLL(name)
        except OSError:
            continue
    return ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))


class _Dim3(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint), ("y", ctypes.c_uint), ("z", ctypes.c_uint)]


class _KParams(ctypes.Structure):  # hipKernelNodeParams
    _fields_ = [("blockDim", _Dim3), ("extra", ctypes.POINTER(ctypes.c_void_p)), ("func", ctypes.c_void_p),
                ("gridDim", _Dim3), ("kernelParams", ctypes.POINTER(ctypes.c_void_p)), ("sharedMemBytes", ctypes.c_uint)]


def _segments():
    """torch allocator segments: (start, end, pool id) -- the graph's private pool vs the default one."""
    out = []
    for seg in torch.cuda.memory_snapshot():
        out.append((seg["address"], seg["address"] + seg["total_size"], tuple(seg.get("segment_pool_id", (0, 0)))))
    return out


def _classify(v: int, segs, user_ptrs):
    for name, (lo, hi) in user_ptrs.items():
        if lo <= v < hi:
            return name
    for lo, hi, pool in segs:
        if lo <= v < hi:
            return "graph_pool" if pool != (0, 0) else "default_pool"
    return "foreign"


def kernel_args(hip, node, segs, user_ptrs):
    """Name of a kernel node and every 8-byte kernel argument word that looks like a device pointer,
    classified by the memory it points into."""
    kp = _KParams()
    if hip.hipGraphKernelNodeGetParams(ctypes.c_void_p(node), ctypes.byref(kp)) != 0:
        return {"error": "params"}
    name = None
    words = []
    ex = kp.extra
    # HIP_LAUNCH_PARAM_BUFFER_POINTER (1), ptr, HIP_LAUNCH_PARAM_BUFFER_SIZE (2), &size, END (3): read only
    # that exact layout (anything else is left alone)
    if ex and ex[0] == 1 and ex[2] == 2 and ex[4] in (None, 3, 0):
        buf = ex[1]
        size = ctypes.cast(ex[3], ctypes.POINTER(ctypes.c_size_t))[0] if ex[3] else 0
        if buf and 0 < size <= 4096:
            words = list((ctypes.c_uint64 * (size // 8)).from_address(buf))
    ptrs = [{"off": 8 * k, "kind": _classify(w, segs, user_ptrs)} for k, w in enumerate(words) if w > (1 << 32)]
    return {"name": name, "grid": [kp.gridDim.x, kp.gridDim.y, kp.gridDim.z], "kernarg_words": len(words),
            "pointers": ptrs, "via": "extra" if kp.extra else ("kernelParams" if kp.kernelParams else None)}


def graph_nodes(graph_handle: int, user_ptrs=None):
    hip = _hip()
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(ctypes.c_void_p(graph_handle), None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(ctypes.c_void_p(graph_handle), nodes, ctypes.byref(n)) == 0
    out = []
    for node in nodes:
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(node), ctypes.byref(t))
        rec = {"type": NODE_TYPES.get(t.value, t.value)}
        if t.value == 0 and user_ptrs is not None:
            rec.update(kernel_args(hip, node, _segments(), user_ptrs))
        if t.value == 1:
            p = _Memcpy3D()
            if hip.hipGraphMemcpyNodeGetParams(ctypes.c_void_p(node), ctypes.byref(p)) == 0:
                a = _PtrAttr()
                rc = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p.srcPtr.ptr))
                hip.hipGetLastError()
                rec.update(kind=p.kind, bytes=p.extent.x * max(1, p.extent.y) * max(1, p.extent.z),
                           src_pageable_host=(rc != 0 or a.type == 0))
        out.append(rec)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--args", default="", help="comma-separated ops whose kernel arguments are classified")
    args = ap.parse_args()
    dev = torch.device("cuda")
    dt = {"bf16": torch.bfloat16, "fp32": torch.float32}[args.dtype]
    torch.manual_seed(0)
    for name, fn, mk_x, mk_dy in cases(dev, dt, args.batch):
        x, dy = mk_x(), mk_dy()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn(x, dy)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g):
            out = fn(x, dy)
        user = None
        if name in args.args.split(","):
            user = {"x": (x.data_ptr(), x.data_ptr() + x.numel() * x.element_size()),
                    "dy": (dy.data_ptr(), dy.data_ptr() + dy.numel() * dy.element_size()),
                    "out": (out.data_ptr(), out.data_ptr() + out.numel() * out.element_size())}
            for d in (fn.__defaults__ or ()):
                if isinstance(d, torch.Tensor):
                    user["w"] = (d.data_ptr(), d.data_ptr() + d.numel() * d.element_size())
        nodes = graph_nodes(g.raw_cuda_graph(), user)
        counts = {}
        for r in nodes:
            counts[r["type"]] = counts.get(r["type"], 0) + 1
        print(json.dumps({"op": name, "dtype": args.dtype, "nodes": counts,
                          "memcpy": [r for r in nodes if r["type"] == "memcpy"],
                          "kernels": [r for r in nodes if r["type"] == "kernel" and "pointers" in r]}), flush=True)
        del g


if __name__ == "__main__":
    main()
