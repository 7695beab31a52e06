"""Does a memset captured into a hipGraph run on every replay?  torch's cross-block row reduction
(sum over dim 0 of a [512, 1000] bf16 tensor) resets its semaphores with hipMemsetAsync; its graph
replays right once and stale from the second replay on (linear_graph_ops.py).

Captured: hipMemsetAsync(t, 0) then t += 1 (a kernel).  Every replay must leave t == 1.  "fixed":
the same capture kept (keep_graph=True), its memset nodes rewritten into fill-kernel nodes by
det_graph_fix_memsets (ops/csrc/det_graph.hip), then instantiated.  Last: torch's sum over dim 0 of
a [512, 1000] bf16 tensor (a cross-block reduction that resets semaphores with a memset), as
captured and fixed, three replays on new inputs.
    python scripts/dbg/memset_graph_repro.py"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _hip():
    for name in ("libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"):
        try:
            return ctypes.CDLL(name)
        except OSError:
            continue
    return ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))


def _fix(g: "torch.cuda.CUDAGraph") -> int:
    from determined_1_amd.ops import _lib

    n = _lib.get_lib().det_graph_fix_memsets(g.raw_cuda_graph(), 1)
    g.instantiate()
    return n


def case(nbytes: int, replays: int = 4, d32: bool = False, fixed: bool = False) -> dict:
    hip = _hip()
    n = nbytes // 4
    t = torch.zeros(n, dtype=torch.int32, device="cuda")
    g = torch.cuda.CUDAGraph(keep_graph=fixed)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        t.add_(1)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        if d32:
            rc = hip.hipMemsetD32Async(ctypes.c_void_p(t.data_ptr()), ctypes.c_int(0), ctypes.c_size_t(n), st)
        else:
            rc = hip.hipMemsetAsync(ctypes.c_void_p(t.data_ptr()), ctypes.c_int(0), ctypes.c_size_t(nbytes), st)
        t.add_(1)
    nfix = _fix(g) if fixed else None
    vals = []
    for _ in range(replays):
        g.replay()
        torch.cuda.synchronize()
        vals.append([int(t.min()), int(t.max())])
    return {"bytes": nbytes, "d32": d32, "fixed": fixed, "memset_nodes": nfix, "rc": rc,
            "after_each_replay_min_max": vals}


def rowsum(fixed: bool, bs: int = 512, replays: int = 3) -> dict:
    torch.manual_seed(0)
    st = torch.randn(bs, 1000, device="cuda", dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        st.sum(0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph(keep_graph=fixed)
    with torch.cuda.graph(g):
        out = st.sum(0)
    nfix = _fix(g) if fixed else None
    res = {"case": f"sum0 [{bs},1000] bf16", "fixed": fixed, "memset_nodes": nfix}
    for k in range(replays):
        new = torch.randn(bs, 1000, device="cuda", dtype=torch.bfloat16)
        ref = new.sum(0)
        st.copy_(new)
        g.replay()
        torch.cuda.synchronize()
        res[f"rel{k}"] = float((out.float() - ref.float()).abs().max() / ref.float().abs().max())
    return res


def main() -> None:
    for nbytes in (4, 16, 256, 4096, 16384, 65536, 262144, 1 << 20):
        for d32 in (False, True):
            print(json.dumps(case(nbytes, d32=d32)), flush=True)
    for nbytes in (4, 16, 4096, 65536, 1 << 20):
        for d32 in (False, True):
            print(json.dumps(case(nbytes, d32=d32, fixed=True)), flush=True)
    for fixed in (False, True):
        print(json.dumps(rowsum(fixed)), flush=True)


if __name__ == "__main__":
    main()
