"""HBM streaming yardstick (det_stream.hip): the best read / write / copy bandwidth the chip sustains,
per buffer size, and the FETCH_SIZE / WRITE_SIZE calibration on known byte counts.

    python scripts/bench_stream.py --sweep [--out gpurun_out/stream.jsonl]
    python scripts/bench_stream.py --calib     # under rocprofv3 --pmc FETCH_SIZE (or WRITE_SIZE)

Sweep: sizes 64 MiB .. 4 GiB; for each, kinds {read (nt / plain loads), write (plain / nt stores),
copy (plain / nt stores)} x unroll {2, 4, 8} x grid {2048, 4096, 8192} workgroups of 256 threads;
the buffer is rewritten by a fill before every timed launch (as a producer kernel leaves its
output), 5 timed launches, the median kept, the best configuration reported per (kind, size).
Read-after-write of a buffer smaller than the 256 MiB Infinity Cache is served partly on-die, so
the small sizes are the cache-assisted ceiling and the >= 1 GiB sizes the HBM ceiling.

Calib: one launch each of a 2 GiB read and a 2 GiB write with fixed configs, separated by
synchronisations, so rocprofv3's per-dispatch FETCH_SIZE / WRITE_SIZE can be compared with the
bytes the kernel must move (the README round-4 claim "FETCH_SIZE is half of a 16-B/lane stream").
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from determined_1_amd.ops import _lib  # noqa: E402

KINDS = {"read_nt": 0, "read": 5, "write": 1, "write_nt": 2, "copy": 3, "copy_nt": 4}


def run(lib, kind, a, b, nbytes, blocks, unroll, sink):
    st = torch.cuda.current_stream().cuda_stream
    rc = lib.det_stream(st, KINDS[kind], a.data_ptr(), b.data_ptr(), nbytes, blocks, unroll, 7, sink.data_ptr())
    _lib.check(rc, "det_stream")


def measure(lib, kind, nbytes, blocks, unroll, bufs, iters=5):
    a, b, sink = bufs
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(iters + 1):
        a.view(torch.int32)[: nbytes // 4].fill_(1)  # freshly written source / destination lines
        e0.record()
        run(lib, kind, a, b, nbytes, blocks, unroll, sink)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = statistics.median(ts[1:])
    moved = nbytes * (2 if kind.startswith("copy") else 1)
    return moved / (ms * 1e-3) / 1e12, ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--calib", action="store_true")
    ap.add_argument("--out", default="")
    ap.add_argument("--max-gib", type=float, default=4.0)
    args = ap.parse_args()
    lib = _lib.get_lib()
    dev = torch.device("cuda")
    cap = int(args.max_gib * (1 << 30))
    a = torch.empty(cap // 4, dtype=torch.int32, device=dev)
    b = torch.empty(cap // 4, dtype=torch.int32, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    if args.calib:
        n = 2 << 30
        for kind in ("read", "write", "copy"):
            a.fill_(1)
            torch.cuda.synchronize()
            run(lib, kind, a, b, n, 8192, 4, sink)
            torch.cuda.synchronize()
            print(json.dumps({"calib": kind, "bytes_read": n if kind != "write" else 0,
                              "bytes_written": n if kind != "read" else 0}), flush=True)
        return
    out = open(args.out, "w") if args.out else None
    sizes = [s << 20 for s in (64, 128, 256, 512, 1024, 2048, 4096) if (s << 20) <= cap]
    best = {}
    for nbytes in sizes:
        for kind in KINDS:
            for unroll in (2, 4, 8):
                for blocks in (2048, 4096, 8192):
                    tbs, ms = measure(lib, kind, nbytes, blocks, unroll, (a, b, sink))
                    rec = {"kind": kind, "MiB": nbytes >> 20, "unroll": unroll, "blocks": blocks, "TBps": round(tbs, 3),
                           "ms": round(ms, 4)}
                    if out:
                        out.write(json.dumps(rec) + "\n")
                    k = (kind, nbytes >> 20)
                    if k not in best or tbs > best[k]["TBps"]:
                        best[k] = rec
            print(json.dumps(best[(kind, nbytes >> 20)]), flush=True)
    if out:
        for rec in best.values():
            out.write(json.dumps(dict(rec, best=True)) + "\n")
        out.close()


if __name__ == "__main__":
    main()
