"""North-star benchmark: ResNet-50 PyTorchTrial training throughput (samples/sec, whole node).

    python bench.py --gpus N --steps K --warmup W     # self-launches N ranks (one per GPU)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Launch (reference: ``harness/determined/horovod.py:124-163`` builds a ``horovodrun -np N``
command, ``layers/_worker_process.py:165-184`` runs it): when ``--gpus N > 1`` and no launcher
env is present, this process becomes a pure launcher -- it makes NO GPU call (torch is not even
imported), spawns N children with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, relays rank 0's JSON
line and exits with the first failing child's code.  Each child binds ``cuda:<local_rank>`` and
joins ProcessGroupNCCL (= RCCL over xGMI).  MIOpen's find database is seeded from the tuned copy
shipped in-tree (``determined_1_amd/ops/miopen_db.py``) so N ranks do not re-tune concurrently.

The step that is timed is the real framework path, not a bare loop: a ``PyTorchTrialController``
is built exactly as a cluster trial process builds it and fed ``RUN_STEP`` workloads:
  warmup RUN_STEP(W batches) -> barrier + synchronize -> t0 -> RUN_STEP(K batches)
  -> synchronize + barrier -> t1.
Each batch is: synthetic uint8 ImageNet-shape images DMA'd from pinned memory -> HIP normalize
kernel -> ResNet-50 fwd/bwd (bf16 autocast, channels_last; the conv weight gradients on a side HIP
stream beside the input-gradient chain) -> [RCCL bucketed all-reduce overlapped with backward] ->
fused arena SGD-momentum HIP kernel.  Weak scaling: fixed per-GPU batch (1,024 by default).

Rank 0 prints ONE JSON line; ``value`` = K * global_batch / max-over-ranks(t1 - t0).

HIP runtime setting: kernel arguments are placed in device memory (``HIP_FORCE_DEV_KERNARG=1``, set
here before anything initialises HIP, inherited by the ranks) -- this step is GPU-bound with ~290
launches, and each kernel then fetches its arguments from HBM instead of host memory over PCIe:
12,470-12,478 vs 12,277-12,280 samples/s in three alternating same-box runs each
(``profiles/r5_bench_resnet50_kernarg_ab.jsonl``).  A host-bound eager step loses with it (BERT
eager 1,159-1,272 vs 1,410-1,414: the host writes every launch's arguments across PCIe), so it is
a per-workload choice, not a framework default.
"""
import argparse
import json
import os
import signal
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")  # see the module docstring

BASELINE_VALUE = None  # BASELINE.json "published": {} -- the reference publishes no ResNet-50 number


def parse() -> argparse.Namespace:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-per-gpu", type=int, default=int(os.environ.get("DET_BENCH_BS", "1024")),
                    help="per-GPU batch (weak scaling).  1024 is the largest whose layer-1 activations stay under "
                         "the kernels' 2 GiB buffer-descriptor range; it peaks at 44.6 GB of the 288 GB HBM and gives "
                         "layer 3/4 (14x14, 7x7) GEMMs enough tiles to fill 256 CUs: 13,53-13,69k vs 13,01-13,09k "
                         "samples/s at 512 (profiles/r6_bench_resnet50_side_stream_batch_sweep.jsonl)")
    ap.add_argument("--amp", default=os.environ.get("DET_BENCH_AMP", "O2"), choices=["O0", "O1", "O2"])
    ap.add_argument("--lr", type=float, default=None,
                    help="SGD learning rate (default: the linear scaling rule, 0.1 x global batch / 256)")
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--image-size", type=int, default=224, help="(smoke tests only; the metric is 224)")
    ap.add_argument("--bucket-mb", type=int, default=int(os.environ.get("DET_BENCH_BUCKET_MB", "64")))
    ap.add_argument("--no-channels-last", action="store_true")
    ap.add_argument("--no-fused-bn", action="store_true", help="stock MIOpen BN + separate add/ReLU (A/B)")
    ap.add_argument("--no-native-conv1x1", action="store_true", help="1x1 convs on MIOpen instead of det_conv GEMMs (A/B)")
    ap.add_argument("--no-native-stem", action="store_true", help="7x7 stem conv on MIOpen instead of det_conv (A/B)")
    ap.add_argument("--no-native-conv3x3", action="store_true", help="3x3 convs on MIOpen instead of det_igemm (A/B)")
    ap.add_argument("--hip-graph", action="store_true",
                    help="1-GPU runs: replay the step from a hipGraph (pytorch/_graph.py; bitwise equal to eager, "
                         "tests/test_graph_memset_gpu.py).  Off by default: the eager step overlaps the conv weight "
                         "gradients on a side stream (ops/arena.py side_work) and that beats the graph replay, which "
                         "runs the two branches one after the other on this runtime (12,96-13,18k vs 12,74-12,89k, "
                         "profiles/r6_wgrad_side_stream_ab.jsonl).  Multi-GPU runs keep DET_STEP_TIMERS on, which "
                         "keeps their steps eager either way")
    ap.add_argument("--no-hip-graph", action="store_true", help="(kept for old command lines: the default now)")
    ap.add_argument("--bn-prologue", action="store_true",
                    help="apply bottleneck bn2 in conv3's GEMM prologue instead of materialising it (A/B)")
    ap.add_argument("--cudnn-benchmark", type=int, default=int(os.environ.get("DET_BENCH_CUDNN_BENCHMARK", "1")),
                    help="MIOpen find mode for the conv algorithms (tuned during the untimed warmup)")
    ap.add_argument("--params-out", default="", help="(verification) save per-tensor float64 sums / norms of the "
                                                     "final parameters to this path")
    ap.add_argument("--launch-timeout", type=float, default=float(os.environ.get("DET_BENCH_LAUNCH_TIMEOUT", "0")),
                    help="self-launch mode: kill all ranks after this many seconds (0 = no limit)")
    return ap.parse_args()


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _miopen_db():
    """``determined_1_amd/ops/miopen_db.py`` loaded by path: importing the package would import
    torch, and the launcher must stay GPU-free."""
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "_det_miopen_db", os.path.join(REPO, "determined_1_amd", "ops", "miopen_db.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # type: ignore
    return mod


def self_launch(args: argparse.Namespace) -> int:
    """Spawn ``args.gpus`` ranks of this script (one process per GPU) and relay rank 0's output.

    The parent never initialises the GPU: it only forks children (no exec of itself), so a
    child's HIP context is the only one on its device.  Children run in their own process group
    so a failure (or the launch timeout) tears the whole job down."""
    miopen_db = _miopen_db()
    n = args.gpus
    port = _free_port()
    base = dict(os.environ)
    procs = []
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DET_BENCH_CHILD="1")
        miopen_db.configure(env)  # a db copy per rank (ranks never share a writable MIOpen db)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      start_new_session=True))

    out_lines = []

    def pump() -> None:
        assert procs[0].stdout is not None
        for raw in procs[0].stdout:
            line = raw.decode(errors="replace")
            out_lines.append(line)
            sys.stdout.write(line)
            sys.stdout.flush()

    t = threading.Thread(target=pump, daemon=True)
    t.start()
    deadline = time.time() + args.launch_timeout if args.launch_timeout > 0 else None
    rc = 0
    live = list(range(n))
    while live:
        for r in list(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.remove(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print(f"bench.py: rank {r} exited with {c}; stopping the other ranks", file=sys.stderr, flush=True)
                for q in procs:
                    if q.poll() is None:
                        try:
                            os.killpg(q.pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
        if deadline is not None and time.time() > deadline and live:
            print(f"bench.py: launch timeout {args.launch_timeout}s; killing ranks {live}", file=sys.stderr, flush=True)
            for r in live:
                try:
                    os.killpg(procs[r].pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
            rc = rc or 124
            deadline = None
        time.sleep(0.2)
    t.join(timeout=10)
    return rc


def main() -> None:
    args = parse()
    launched = "WORLD_SIZE" in os.environ
    if not launched and args.gpus > 1:
        sys.exit(self_launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: launcher started {world} ranks but --gpus is {args.gpus}", file=sys.stderr)
        sys.exit(2)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if os.environ.get("DET_BENCH_CHILD") != "1":
        _miopen_db().configure(os.environ)
    if world > 1:
        # phase timers (forward / backward / exposed comm / optimizer) on every multi-GPU run: DP
        # steps are never hipGraph-captured, so the events add no synchronisation to the path
        os.environ.setdefault("DET_STEP_TIMERS", "1")
    import torch

    torch.backends.cudnn.benchmark = bool(args.cudnn_benchmark)

    from determined_1_amd import workload
    from determined_1_amd.experimental import make_controller
    from determined_1_amd.experimental import load_model_def

    ResNetImageNetTrial = load_model_def(os.path.join(REPO, "examples", "computer_vision", "resnet50_pytorch")).ResNetImageNetTrial
    from determined_1_amd.parallel import dist as pdist

    gbs = args.batch_per_gpu * world
    config = {
        "entrypoint": "model_def:ResNetImageNetTrial",
        "hyperparameters": {
            "global_batch_size": gbs,
            "lr": args.lr if args.lr is not None else 0.1 * gbs / 256,
            "momentum": 0.9,
            "weight_decay": 5e-5,
            "arch": args.arch,
            "amp": args.amp,
            "channels_last": not args.no_channels_last,
            "fused_bn": not args.no_fused_bn,
            "native_conv1x1": not args.no_native_conv1x1,
            "bn_prologue": args.bn_prologue,
            "native_stem": not args.no_native_stem,
            "native_conv3x3": not args.no_native_conv3x3,
            "image_size": args.image_size,
        },
        "resources": {"slots_per_trial": world},
        "optimizations": {"tensor_fusion_threshold": args.bucket_mb, "hip_graph": world == 1 and args.hip_graph and not args.no_hip_graph},
        "searcher": {"name": "single", "metric": "validation_loss", "max_length": {"batches": args.steps}},
        "scheduling_unit": args.steps,
    }
    timing = {}

    def sync_barrier() -> None:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        pdist.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def stream():
        resp = {}

        def keep(r):
            resp["last"] = r

        # warmup one batch per workload so the time to each completed batch is visible (MIOpen
        # find/compile cost lands in the first batches; the rest is steady state)
        for i in range(args.warmup):
            yield workload.train_workload(1, num_batches=1, total_batches_processed=i), [], keep
            timing.setdefault("warm", []).append(round(time.perf_counter() - t_start, 2))
            if rank == 0:
                print(f"[bench rank0] warmup batch {i + 1}/{args.warmup} done at {timing['warm'][-1]:.1f}s",
                      file=sys.stderr, flush=True)
        sync_barrier()
        timing["t0"] = time.perf_counter()
        yield workload.train_workload(2, num_batches=args.steps, total_batches_processed=args.warmup), [], keep
        sync_barrier()
        timing["t1"] = time.perf_counter()
        timing["resp"] = resp.get("last")
        yield workload.terminate_workload(3), [], workload.ignore_response

    if torch.cuda.is_available():
        torch.cuda.set_device(pdist.local_cuda_device(local_rank))
    t_start = time.perf_counter()

    def heartbeat() -> None:  # MIOpen find mode can run minutes in warmup with no other output
        while True:
            time.sleep(30)
            phase = "timed" if "t0" in timing else "warmup"
            print(f"[bench rank{rank}] {phase} {time.perf_counter() - t_start:.0f}s", file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    ctrl = make_controller(ResNetImageNetTrial, config, stream(), trial_seed=1234)
    timing["ctrl_built"] = time.perf_counter()
    ctrl.run()
    from determined_1_amd.ops import arena

    side_wgrad = {"on": arena.SIDE_WGRAD, **arena.SIDE_COUNTS}
    if args.params_out and int(os.environ.get("RANK", "0")) == 0:
        ps = [p.detach().double() for p in ctrl.context.models[0].parameters()]
        torch.save({"sums": torch.stack([p.sum() for p in ps]).cpu(), "norms": torch.stack([p.norm() for p in ps]).cpu(),
                    "graph": getattr(getattr(ctrl, "_graph", None), "stats", lambda: None)()}, args.params_out)
    elapsed = timing["t1"] - timing["t0"]
    warmup_s = timing["t0"] - t_start
    import torch.distributed as tdist

    seen = (tdist.get_world_size(), tdist.get_backend()) if tdist.is_initialized() else (1, None)
    phases = getattr(ctrl, "last_step_timers", None) or {}
    per_rank = pdist.allgather_object((elapsed, warmup_s, seen[0], seen[1], phases))
    t = max(e[0] for e in per_rank)
    value = args.steps * gbs / t
    loss = None
    r = timing.get("resp")
    if isinstance(r, dict):
        loss = r.get("metrics", {}).get("avg_metrics", {}).get("loss")
    if rank == 0:
        out = {
            "metric": "samples/sec (whole node) ResNet-50 PyTorchTrial",
            "value": round(value, 2),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * t / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": "bf16" if args.amp != "O0" else "fp32",
            "data": f"synthetic (random uint8 {args.image_size}x{args.image_size}x3 images, random labels; random-init weights)",
            "config": {
                "model": args.arch,
                "global_batch": gbs,
                "per_gpu_batch": args.batch_per_gpu,
                "seq_len": None,
                "image_size": args.image_size,
                "parallelism": f"dp{world}",
                "amp": args.amp,
                "optimizer": "SGD-momentum (fused arena HIP kernel)",
                "bucket_mb": args.bucket_mb,
                "fused_bn": not args.no_fused_bn,
                "native_conv1x1": not args.no_native_conv1x1,
                "bn_prologue": args.bn_prologue,
                "native_stem": not args.no_native_stem,
                "native_conv3x3": not args.no_native_conv3x3,
                "final_avg_loss": loss,
                "world_size_seen": [e[2] for e in per_rank],
                "backend": per_rank[0][3],
                "warmup_s": round(max(e[1] for e in per_rank), 1),
                "warmup_batch_done_s": timing.get("warm"),
                "startup_s": round(timing.get("ctrl_built", 0.0) - t_start, 1),
                "miopen_find_db": os.environ.get("MIOPEN_USER_DB_PATH"),
                "hip_graph": getattr(getattr(ctrl, "_graph", None), "stats", lambda: None)(),
                "wgrad_side_stream": side_wgrad,
                "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1) if torch.cuda.is_available() else None,
            },
        }
        if phases:  # DET_STEP_TIMERS=1: per-batch device phases of the timed window (forward/backward/comm/opt)
            out["config"]["phase_ms"] = {k.split("/", 1)[1]: round(v, 3) for k, v in phases.items()}
        if world > 1:
            steps_ms = [1000.0 * e[0] / args.steps for e in per_rank]
            out["config"]["rank_ms_per_step"] = [round(x, 3) for x in steps_ms]
            out["config"]["rank_skew_pct"] = round(100.0 * (max(steps_ms) - min(steps_ms)) / max(steps_ms), 2)
            exposed = [e[4].get("timer/comm_exposed_ms") for e in per_rank if e[4]]
            if exposed:
                out["config"]["rank_comm_exposed_ms"] = [round(x, 3) for x in exposed]
        print(json.dumps(out), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
