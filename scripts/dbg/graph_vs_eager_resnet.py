"""Per-step parameter trace of the ResNet trial, eager or hipGraph (DET_HIP_GRAPH=0/1), for
finding the first step and tensor where a replayed step departs from the eager one.

  python scripts/dbg/graph_vs_eager_resnet.py --out A.pt [--steps 12 --bs 64 --image 64]
  python scripts/dbg/graph_vs_eager_resnet.py --compare A.pt B.pt

Records after every batch: every parameter (float64 copy of the small ones, sums/norms of all),
the gradient the optimizer consumed (``p.grad`` as the harness leaves it) and the loss.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def run(args: argparse.Namespace) -> None:
    import torch

    from determined_1_amd import workload
    from determined_1_amd.experimental import load_model_def, make_controller

    trial_cls = load_model_def(os.path.join(REPO, "examples", "computer_vision", "resnet50_pytorch")).ResNetImageNetTrial
    config = {
        "entrypoint": "model_def:ResNetImageNetTrial",
        "hyperparameters": {"global_batch_size": args.bs, "lr": 0.1 * args.bs / 256, "momentum": 0.9,
                            "weight_decay": 5e-5, "arch": args.arch, "amp": "O2", "channels_last": True,
                            "image_size": args.image},
        "resources": {"slots_per_trial": 1},
        "searcher": {"name": "single", "metric": "validation_loss", "max_length": {"batches": args.steps}},
        "scheduling_unit": 1,
    }
    rec = {"params": [], "grads": [], "loss": [], "names": None}
    holder = {}

    # --one-workload W: W one-batch workloads (bench.py's warmup) then the remaining steps as ONE
    # workload (no host synchronisation between its batches), recording only after each workload
    plan = [(i, 1) for i in range(args.steps)] if args.one_workload <= 0 else \
        [(i, 1) for i in range(args.one_workload)] + [(args.one_workload, args.steps - args.one_workload)]

    def stream():
        for wi, (start, nb) in enumerate(plan):
            yield workload.train_workload(wi + 1, num_batches=nb, total_batches_processed=start), [], \
                lambda r: rec["loss"].append(r)
            ctrl = holder["ctrl"]
            m = ctrl.context.models[0]
            named = list(m.named_parameters())
            rec["names"] = [n for n, _ in named]
            rec["params"].append([p.detach().double().cpu() if p.numel() <= 4096 else
                                  torch.stack([p.detach().double().sum(), p.detach().double().norm()]).cpu()
                                  for _, p in named])
            rec["grads"].append([None if p.grad is None else
                                 (p.grad.detach().double().cpu() if p.numel() <= 4096 else
                                  torch.stack([p.grad.detach().double().sum(), p.grad.detach().double().norm()]).cpu())
                                 for _, p in named])
            # the arena gradient slots (a fresh window overwrites them; they keep the last step's
            # gradient) and the arena params of every 1-D [num_classes] tensor (fc.bias)
            small = []
            for st in ctrl.context._opt_states:
                sink = getattr(st.fused, "sink", None) if st.fused is not None else None
                for a, idx in (sink.groups if sink is not None else []):
                    for i in idx:
                        if tuple(a.params[i].shape) == (1000,):
                            small.append((a.grad_views[i].detach().double().cpu(), a.params[i].detach().double().cpu()))
            rec.setdefault("fcb", []).append(small)
        yield workload.terminate_workload(args.steps + 1), [], workload.ignore_response

    if args.trace_sink:
        _trace_sink(rec)
    torch.cuda.set_device(0)
    holder["ctrl"] = make_controller(trial_cls, config, stream(), trial_seed=1234)
    holder["ctrl"].run()
    g = getattr(holder["ctrl"], "_graph", None)
    rec["graph"] = g.stats() if g is not None else None
    if args.dump_nodes and g is not None:  # needs DET_GRAPH_KEEP=1
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from graph_nodes import graph_nodes

        for key, cg in g.graphs.items():
            nodes = graph_nodes(cg.graph.raw_cuda_graph())
            counts = {}
            for r in nodes:
                counts[r["type"]] = counts.get(r["type"], 0) + 1
            print("graph nodes", counts, flush=True)
            for k, r in enumerate(nodes):
                if r["type"] not in ("kernel", "empty"):
                    print("  node", k, r, flush=True)
    rec["loss"] = [repr(x)[:200] for x in rec["loss"]]
    torch.save(rec, args.out)
    print("saved", args.out, rec["graph"], flush=True)
    for e in rec.get("sink_log", []):
        print(e)


def _trace_sink(rec: dict) -> None:
    """Log what the GradSink does with the fc-layer gradients (shapes [1000] / [1000, 2048])."""
    import torch

    from determined_1_amd.ops import arena

    log = rec.setdefault("sink_log", [])
    hook0, flush0, end0 = arena.GradSink._hook, arena.GradSink._flush, arena.GradSink.end_backward

    def hook(self, p):
        if tuple(p.shape) in ((1000,), (1000, 2048)):
            slot = self._slot.get(id(p))
            g = p.grad
            log.append(("hook", tuple(p.shape), self.fresh, torch.cuda.is_current_stream_capturing(),
                        None if g is None else (g.dtype == slot[7], tuple(g.stride()) == tuple(slot[6]),
                                                g.data_ptr() == slot[4], g is slot[3]),
                        slot[0], self._pending[slot[0]]))
        return hook0(self, p)

    def flush(self, gi):
        shapes = [tuple(g.shape) for _, g in self._stolen[gi]]
        log.append(("flush", gi, len(shapes), [s for s in shapes if s in ((1000,), (1000, 2048))],
                    torch.cuda.is_current_stream_capturing()))
        return flush0(self, gi)

    def end(self):
        log.append(("end_backward", self.fresh, list(self._pending)))
        return end0(self)

    arena.GradSink._hook, arena.GradSink._flush, arena.GradSink.end_backward = hook, flush, end


def compare(a_path: str, b_path: str) -> None:
    import torch

    a, b = torch.load(a_path, weights_only=True), torch.load(b_path, weights_only=True)
    names = a["names"]
    print("graph:", b.get("graph"))
    for step, (pa, pb, ga, gb) in enumerate(zip(a["params"], b["params"], a["grads"], b["grads"])):
        worst = []
        for i, (x, y) in enumerate(zip(pa, pb)):
            d = float((x - y).abs().max() / (y.abs().max() + 1e-12))
            worst.append((d, names[i], "param"))
        for i, (x, y) in enumerate(zip(ga, gb)):
            if x is None or y is None:
                if (x is None) != (y is None):
                    worst.append((float("inf"), names[i], f"grad None a={x is None} b={y is None}"))
                continue
            d = float((x - y).abs().max() / (y.abs().max() + 1e-12))
            worst.append((d, names[i], "grad"))
        worst.sort(key=lambda t: -t[0])
        print(f"step {step}: " + "; ".join(f"{n} {k} {d:.3g}" for d, n, k in worst[:5]))
    fa, fb = a["params"][-1][-1], b["params"][-1][-1]
    print("last param a[:8]", fa.flatten()[:8].tolist())
    print("last param b[:8]", fb.flatten()[:8].tolist())


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--compare", nargs=2, default=None)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--bs", type=int, default=64)
    ap.add_argument("--image", type=int, default=64)
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--one-workload", type=int, default=0)
    ap.add_argument("--trace-sink", action="store_true")
    ap.add_argument("--dump-nodes", action="store_true")
    args = ap.parse_args()
    if args.compare:
        compare(*args.compare)
    else:
        run(args)


if __name__ == "__main__":
    main()
