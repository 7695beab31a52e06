"""Which library op mis-replays inside a multi-step hipGraph?  (Round-5 finding: the CIFAR trial's
torch layers at bf16 go non-finite only in 20-step chunk graphs -- without dropout too -- while fp32
(O0), per-batch graphs, eager and the native CNN kernels stay clean.)

For each op of the CIFAR network (bf16, channels_last, batch 32) it captures K calls on K distinct
preallocated inputs into ONE graph, replays it R times, and compares every replay's outputs with
the eager results of the same calls: a correct replay matches eager up to the op's own run-to-run
nondeterminism (measured as eager vs eager).

    python scripts/dbg/miopen_graph_repro.py --k 20 --replays 5 [--deterministic]
"""
import argparse
import json

import torch
import torch.nn.functional as F


def _maybe_fix(args, g) -> None:
    """--fix-memsets: rewrite the captured memset nodes into fill-kernel nodes (ops/csrc/det_graph.hip;
    the HIP runtime's small captured memsets replay a stale value, memset_graph_repro.py)."""
    if not args.fix_memsets:
        return
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from determined_1_amd.ops import _lib

    n = _lib.get_lib().det_graph_fix_memsets(g.raw_cuda_graph(), 1)
    print(json.dumps({"memset_nodes_rewritten": n}), flush=True)
    g.instantiate()


def cases(dev, dt, n):
    cl = torch.channels_last
    convs = [("conv1", 3, 32, 32, 0), ("conv2", 32, 32, 30, 0), ("conv3", 32, 64, 14, 1), ("conv4", 64, 64, 14, 0)]
    out = []
    for name, ci, co, hw, pad in convs:
        w = (torch.randn(co, ci, 3, 3, device=dev) * 0.1).to(dt).contiguous(memory_format=cl)
        ho = hw + 2 * pad - 2

        def mk_x(ci=ci, hw=hw):
            return torch.randn(n, ci, hw, hw, device=dev).to(dt).contiguous(memory_format=cl)

        def mk_dy(co=co, ho=ho):
            return torch.randn(n, co, ho, ho, device=dev).to(dt).contiguous(memory_format=cl)

        out.append((f"{name}_fwd", lambda x, dy, w=w, pad=pad: F.conv2d(x, w, padding=pad), mk_x, mk_dy))
        out.append((f"{name}_bwd_data", lambda x, dy, w=w, pad=pad: torch.ops.aten.convolution_backward(
            dy, x, w, [w.shape[0]], [1, 1], [pad, pad], [1, 1], False, [0, 0], 1, [True, False, False])[0], mk_x, mk_dy))
        out.append((f"{name}_bwd_weight", lambda x, dy, w=w, pad=pad: torch.ops.aten.convolution_backward(
            dy, x, w, [w.shape[0]], [1, 1], [pad, pad], [1, 1], False, [0, 0], 1, [False, True, True])[1], mk_x, mk_dy))
    for name, i, o in (("fc1", 2304, 512), ("fc2", 512, 10)):
        w = (torch.randn(o, i, device=dev) * 0.05).to(dt)

        def mk_x(i=i):
            return torch.randn(n, i, device=dev).to(dt)

        def mk_dy(o=o):
            return torch.randn(n, o, device=dev).to(dt)

        out.append((f"{name}_fwd", lambda x, dy, w=w: F.linear(x, w), mk_x, mk_dy))
        out.append((f"{name}_dgrad", lambda x, dy, w=w: dy @ w, mk_x, mk_dy))
        out.append((f"{name}_wgrad", lambda x, dy, w=w: dy.t() @ x, mk_x, mk_dy))

    def mk_p():
        return torch.randn(n, 32, 28, 28, device=dev).to(dt).contiguous(memory_format=cl)

    def pool_bwd(x, dy):
        y, idx = F.max_pool2d_with_indices(x, 2)
        return torch.ops.aten.max_pool2d_with_indices_backward(dy, x, [2, 2], [2, 2], [0, 0], [1, 1], False, idx)

    out.append(("maxpool_bwd", pool_bwd, mk_p,
                lambda: torch.randn(n, 32, 14, 14, device=dev).to(dt).contiguous(memory_format=cl)))
    return out


def clobber(args, dev):
    """Release every cached block to the driver and refill device memory with NaN-filled tensors:
    a graph node that kept a pointer to memory its pool does not own (freed during capture) now
    reads NaN there -- and writes into these buffers, which ``clobbered`` counts afterwards."""
    if not args.clobber:
        return []
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    bufs = []
    for _ in range(args.clobber):
        b = torch.empty(256 << 20, dtype=torch.float32, device=dev)  # 1 GiB each
        b.fill_(float("nan"))
        bufs.append(b)
    torch.cuda.synchronize()
    return bufs


def poison_cache(dev, gib=16):
    """Leave NaN in the allocator's cached blocks: the next allocations hand out NaN-filled memory,
    so an op that reads its output (or a workspace) before writing it shows up as non-finite."""
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    bufs = [torch.empty(256 << 20, dtype=torch.float32, device=dev).fill_(float("nan")) for _ in range(gib)]
    torch.cuda.synchronize()
    del bufs  # back into the cache, still NaN


def poison_mode(args, dev, dt):
    """Eager only: every op (and whole steps) once on a clean cache and once on a NaN-poisoned one."""
    torch.manual_seed(0)
    for name, fn, mk_x, mk_dy in cases(dev, dt, args.batch):
        if args.only and name not in args.only.split(","):
            continue
        x, dy = mk_x(), mk_dy()
        ref = fn(x, dy).float().clone()
        poison_cache(dev)
        out = fn(x, dy).float()
        print(json.dumps({"op": name, "poisoned_nonfinite": int((~torch.isfinite(out)).sum()),
                          "max_abs": float((out - ref).abs().nan_to_num(float("inf")).max()),
                          "scale": float(ref.abs().max())}), flush=True)


def clobbered(bufs):
    return int(sum(int((~torch.isnan(b)).sum()) for b in bufs))


def step_mode(args, dev, dt):
    """The whole CIFAR step (torch layers, no dropout, SGD) K times in one graph vs eager K steps."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from determined_1_amd.models import CIFAR10CNN

    torch.manual_seed(0)
    if args.arch == "cnn":
        model = CIFAR10CNN(0.0, 0.0, 0.0).to(dev).to(memory_format=torch.channels_last).to(dt)
        model.native = False
    elif args.arch == "mlp":  # linear layers only (hipBLASLt / rocBLAS), no convolutions
        model = torch.nn.Sequential(torch.nn.Flatten(), torch.nn.Linear(3072, 2304), torch.nn.ReLU(),
                                    torch.nn.Linear(2304, 512), torch.nn.ReLU(), torch.nn.Linear(512, 10)).to(dev).to(dt)
    else:  # convolutions only (MIOpen), the head a global average pool
        model = torch.nn.Sequential(torch.nn.Conv2d(3, 32, 3), torch.nn.ReLU(), torch.nn.Conv2d(32, 32, 3), torch.nn.ReLU(),
                                    torch.nn.MaxPool2d(2), torch.nn.Conv2d(32, 64, 3, padding=1), torch.nn.ReLU(),
                                    torch.nn.Conv2d(64, 10, 3), torch.nn.AdaptiveAvgPool2d(1), torch.nn.Flatten())
        model = model.to(dev).to(memory_format=torch.channels_last).to(dt)
    params = list(model.parameters())
    xs = [torch.randn(args.batch, 3, 32, 32, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
          for _ in range(args.k)]
    ys = [torch.randint(0, 10, (args.batch,), device=dev) for _ in range(args.k)]
    lr = 0.01

    if args.grads == "zero":
        for p in params:
            p.grad = torch.zeros_like(p)

    def steps():
        losses = []
        for x, y in zip(xs, ys):
            loss = F.cross_entropy(model(x).float(), y)
            loss.backward()
            with torch.no_grad():
                for p in params:
                    if args.update == "sub":
                        p.sub_(lr * p.grad)
                    if args.grads == "none":
                        p.grad = None
                    else:
                        p.grad.zero_()
            losses.append(loss.detach())
        return torch.stack(losses)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        steps()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph(keep_graph=args.fix_memsets)
    with torch.cuda.graph(g):
        static = steps()
    _maybe_fix(args, g)
    for r in range(args.replays):
        start = [p.detach().clone() for p in params]
        bufs = clobber(args, dev)
        g.replay()
        torch.cuda.synchronize()
        written = clobbered(bufs)
        del bufs
        lg = static.clone()
        pg = [p.detach().clone() for p in params]
        if args.no_eager:
            print(json.dumps({"mode": "step", "replay": r, "graph_losses_finite": bool(torch.isfinite(lg).all()),
                              "loss_first_last": [float(lg[0]), float(lg[-1])],
                              "foreign_writes": written if args.clobber else None}), flush=True)
            continue
        with torch.no_grad():
            for p, v in zip(params, start):
                p.copy_(v)
        if args.poison_steps:
            poison_cache(dev)
        le = steps()
        torch.cuda.synchronize()
        pe = [p.detach().clone() for p in params]
        d = max(float((a.float() - b.float()).abs().max()) for a, b in zip(pg, pe))
        print(json.dumps({"mode": "step", "replay": r, "graph_losses_finite": bool(torch.isfinite(lg).all()),
                          "first_nonfinite": int((~torch.isfinite(lg)).nonzero()[0]) if not torch.isfinite(lg).all() else None,
                          "loss_max_abs": float((lg - le).abs().max()), "param_max_abs": d,
                          "foreign_writes": written if args.clobber else None,
                          "deterministic": args.deterministic}), flush=True)
        with torch.no_grad():  # continue from the graph's result
            for p, v in zip(params, pg):
                p.copy_(v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--replays", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--deterministic", action="store_true")
    ap.add_argument("--step", action="store_true", help="whole training steps instead of single ops")
    ap.add_argument("--fix-memsets", action="store_true", help="rewrite captured memset nodes (det_graph.hip)")
    ap.add_argument("--clobber", type=int, default=0,
                    help="GiB of NaN-filled memory allocated after empty_cache() before every replay")
    ap.add_argument("--only", default="", help="comma-separated op names (op mode)")
    ap.add_argument("--no-eager", action="store_true", help="step mode: replays only, no eager steps in between")
    ap.add_argument("--poison", action="store_true", help="eager ops on a NaN-poisoned allocator cache")
    ap.add_argument("--arch", default="cnn", choices=("cnn", "mlp", "conv"), help="step mode: the model")
    ap.add_argument("--no-miopen", action="store_true", help="torch.backends.cudnn.enabled = False")
    ap.add_argument("--interleave", action="store_true", help="op mode: eager calls of every op between replays")
    ap.add_argument("--poison-steps", action="store_true", help="step mode: poison the cache before the eager steps")
    ap.add_argument("--update", default="sub", choices=("sub", "none"), help="step mode: SGD update or none")
    ap.add_argument("--grads", default="none", choices=("none", "zero"),
                    help="step mode: grads set to None after each step (allocated in the graph) or zeroed in place")
    args = ap.parse_args()
    torch.backends.cudnn.deterministic = args.deterministic
    if args.no_miopen:
        torch.backends.cudnn.enabled = False
    dev = torch.device("cuda")
    dt = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16}[args.dtype]
    if args.poison:
        return poison_mode(args, dev, dt)
    if args.step:
        return step_mode(args, dev, dt)
    torch.manual_seed(0)
    report = []
    all_cases = cases(dev, dt, args.batch)
    for name, fn, mk_x, mk_dy in all_cases:
        if args.only and name not in args.only.split(","):
            continue
        xs = [mk_x() for _ in range(args.k)]
        dys = [mk_dy() for _ in range(args.k)]
        eager = [fn(x, dy).float() for x, dy in zip(xs, dys)]
        eager2 = [fn(x, dy).float() for x, dy in zip(xs, dys)]
        noise = max(float((a - b).abs().max()) for a, b in zip(eager, eager2))
        scale = max(float(a.abs().max()) for a in eager)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for x, dy in zip(xs, dys):
                fn(x, dy)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph(keep_graph=args.fix_memsets)
        with torch.cuda.graph(g):
            outs = [fn(x, dy) for x, dy in zip(xs, dys)]
        _maybe_fix(args, g)
        worst, nonfinite, first_bad, foreign = 0.0, 0, None, 0
        for r in range(args.replays):
            for o in outs:
                o.fill_(float("nan"))  # a replay that skips a write leaves NaN behind
            bufs = clobber(args, dev)
            g.replay()
            torch.cuda.synchronize()
            foreign += clobbered(bufs)
            del bufs
            if args.interleave:  # eager calls of every op of the network between replays
                for _, fn2, mkx2, mkdy2 in all_cases:
                    fn2(mkx2(), mkdy2())
                torch.cuda.synchronize()
            for i, (o, e) in enumerate(zip(outs, eager)):
                of = o.float()
                if not torch.isfinite(of).all():
                    nonfinite += 1
                    first_bad = first_bad or (r, i)
                    continue
                worst = max(worst, float((of - e).abs().max()))
        row = {"op": name, "eager_noise": noise, "scale": scale, "graph_vs_eager_max": worst,
               "nonfinite_outputs": nonfinite, "first_bad": first_bad, "foreign_writes": foreign,
               "ok": nonfinite == 0 and foreign == 0 and worst <= max(2 * noise, 1e-6 * scale)}
        report.append(row)
        print(json.dumps(row), flush=True)
        del g, outs
    print(json.dumps({"dtype": args.dtype, "k": args.k, "deterministic": args.deterministic,
                      "bad": [r["op"] for r in report if not r["ok"]]}), flush=True)


if __name__ == "__main__":
    main()
