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

    def stream():
        for i in range(args.steps):
            yield workload.train_workload(i + 1, num_batches=1, total_batches_processed=i), [], \
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
        yield workload.terminate_workload(args.steps + 1), [], workload.ignore_response

    torch.cuda.set_device(0)
    holder["ctrl"] = make_controller(trial_cls, config, stream(), trial_seed=1234)
    holder["ctrl"].run()
    g = getattr(holder["ctrl"], "_graph", None)
    rec["graph"] = g.stats() if g is not None else None
    rec["loss"] = [repr(x)[:200] for x in rec["loss"]]
    torch.save(rec, args.out)
    print("saved", args.out, rec["graph"], flush=True)


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
    args = ap.parse_args()
    if args.compare:
        compare(*args.compare)
    else:
        run(args)


if __name__ == "__main__":
    main()
