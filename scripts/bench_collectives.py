"""Collective micro-benchmark for the gradient-reduction paths over RCCL/xGMI (first-contact kit
for an N-GPU node).

    python scripts/bench_collectives.py --gpus N [--sizes-mb 2,4,8,16,32,64] [--iters 20]

Self-launches N ranks like ``bench.py`` (the parent makes no GPU call; ``--gpus 1`` or an
existing WORLD_SIZE runs in-process).  Per bucket size it times, on every rank, in one process:
  * ``allreduce_bf16`` / ``allreduce_fp32``: RCCL all-reduce (what ``grad_reduction: allreduce``
    and fp32 arenas issue);
  * ``fp32_accum_bf16``: all-to-all reduce-scatter + the ``det_sum_rows`` fp32 shard sum +
    all-gather (``grad_reduction: fp32_accum``, ``parallel/ddp.py``);
and reports the MAX over ranks of the median time, the algorithm bandwidth (bytes / t) and the
bus bandwidth 2(N-1)/N x bytes / t (ring-equivalent traffic per GPU), plus bus bandwidth per
xGMI link (/ (N-1): every peer is one point-to-point link on a fully connected node).  Rank 0
prints one JSON line per (size, algorithm) and a final summary with the per-size winner --
the same decision ``grad_reduction: auto`` takes inside a trial.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def parse() -> argparse.Namespace:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--sizes-mb", default="2,4,8,16,32,64")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--backend", default=None, help="default: nccl (RCCL) on GPUs, gloo on CPU")
    ap.add_argument("--cpu", action="store_true", help="gloo on CPU tensors (plumbing check without GPUs)")
    return ap.parse_args()


def self_launch(args: argparse.Namespace) -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    for p in procs:
        c = p.wait()
        rc = rc or c
    return rc


def main() -> None:
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args))
    import torch
    import torch.distributed as dist

    from determined_1_amd.ops.functional import sum_rows_

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        os.environ["MASTER_PORT"] = "29511"
    use_gpu = not args.cpu and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dev = torch.device("cuda") if use_gpu else torch.device("cpu")
    dist.init_process_group(args.backend or ("nccl" if use_gpu else "gloo"), rank=rank, world_size=world)

    def sync() -> None:
        if use_gpu:
            torch.cuda.synchronize()

    def timed(fn) -> float:
        for _ in range(3):
            fn()
        sync()
        dist.barrier()
        ts = []
        for _ in range(args.iters):
            t0 = time.perf_counter()
            fn()
            sync()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        t = torch.tensor([ts[len(ts) // 2]], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    results = []
    for mb in [float(x) for x in args.sizes_mb.split(",") if x]:
        nbytes = int(mb * 1024 * 1024)
        n_bf = (nbytes // 2) // (64 * world) * (64 * world)
        n_f32 = (nbytes // 4) // (64 * world) * (64 * world)
        bf = torch.randn(n_bf, device=dev).to(torch.bfloat16)
        f32 = torch.randn(n_f32, device=dev)
        recv = torch.empty_like(bf)
        shard_n = n_bf // world

        def fp32_accum() -> None:
            shard = bf[rank * shard_n:(rank + 1) * shard_n]
            dist.all_to_all_single(recv, bf)
            sum_rows_(recv, world, shard)
            dist.all_gather_into_tensor(bf, shard)

        algos = {
            "allreduce_bf16": (lambda: dist.all_reduce(bf), n_bf * 2),
            "allreduce_fp32": (lambda: dist.all_reduce(f32), n_f32 * 4),
            "fp32_accum_bf16": (fp32_accum, n_bf * 2),
        }
        for name, (fn, b) in algos.items():
            t = timed(fn)
            bus = 2.0 * (world - 1) / world * b / t if world > 1 else 0.0
            rec = {"size_mb": mb, "algo": name, "world": world, "ms": round(1e3 * t, 4),
                   "algbw_GBs": round(b / t / 1e9, 2), "busbw_GBs": round(bus / 1e9, 2),
                   "busbw_per_link_GBs": round(bus / max(1, world - 1) / 1e9, 2), "backend": dist.get_backend()}
            results.append(rec)
            if rank == 0:
                print(json.dumps(rec), flush=True)
    if rank == 0:
        winners = {}
        for mb in sorted({r["size_mb"] for r in results}):
            ar = next(r for r in results if r["size_mb"] == mb and r["algo"] == "allreduce_bf16")
            fa = next(r for r in results if r["size_mb"] == mb and r["algo"] == "fp32_accum_bf16")
            winners[str(mb)] = "allreduce" if ar["ms"] < 0.9 * fa["ms"] else "fp32_accum"
        print(json.dumps({"summary": "bf16 bucket reduction choice (auto rule: allreduce only if >=10% faster)",
                          "world": world, "choice_by_mb": winners}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
