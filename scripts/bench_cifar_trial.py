"""Per-batch cost of the ASHA benchmark's trial (examples/computer_vision/cifar10_pytorch CIFARTrial)
run through the real PyTorchTrial controller on one GPU: startup phases, train ms/batch and the
validation pass (10k records), at the batch sizes the adaptive.yaml search space draws (16..64).

    python scripts/bench_cifar_trial.py [--batch 32] [--batches 2000] [--amp O2]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(REPO, "examples", "computer_vision", "cifar10_pytorch")
sys.path.insert(0, REPO)
sys.path.insert(0, EX)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--batches", type=int, default=2000)
    ap.add_argument("--chunk", type=int, default=500)
    ap.add_argument("--amp", default="O2")
    ap.add_argument("--hip-graph", action="store_true", help="optimizations.hip_graph: replay train_batch as a hipGraph")
    ap.add_argument("--graph-batches", type=int, default=1, help="optimizations.hip_graph_batches")
    ap.add_argument("--seed", type=int, default=0, help="trial seed")
    ap.add_argument("--lr", type=float, default=1e-3, help="RMSprop learning rate (const.yaml: 1e-4)")
    ap.add_argument("--train-records", type=int, default=50000, help="records per epoch")
    ap.add_argument("--no-dropout", action="store_true", help="dropout 0 (deterministic eager/graph comparison)")
    ap.add_argument("--batch-losses", action="store_true", help="also print every batch's loss")
    ap.add_argument("--validations", type=int, default=1, help="validation passes at the end (the first captures)")
    args = ap.parse_args()
    t0 = time.time()
    import torch

    from determined_1_amd import workload
    from determined_1_amd.experimental import make_controller
    import model_def

    t_import = time.time() - t0
    cfg = {"hyperparameters": {"global_batch_size": args.batch, "learning_rate": args.lr, "train_records": args.train_records, "learning_rate_decay": 1e-6,
                               "layer1_dropout": 0.0 if args.no_dropout else 0.25,
                               "layer2_dropout": 0.0 if args.no_dropout else 0.25,
                               "layer3_dropout": 0.0 if args.no_dropout else 0.5,
                               "amp": args.amp},
           "searcher": {"name": "single", "metric": "validation_error", "max_length": {"batches": args.batches}},
           "records_per_epoch": args.train_records, "scheduling_unit": args.chunk,
           "optimizations": {"hip_graph": bool(args.hip_graph), "hip_graph_batches": args.graph_batches}}
    marks = []
    res = {}

    def keep(name):
        def f(r):
            res[name] = r
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            marks.append((name, time.time()))
        return f

    def stream():
        done = 0
        step = 1
        while done < args.batches:
            n = min(args.chunk, args.batches - done)
            yield workload.train_workload(step, num_batches=n, total_batches_processed=done), [], keep(f"train{step}")
            done += n
            step += 1
        for v in range(args.validations):
            yield workload.validation_workload(step, total_batches_processed=done), [], keep("val" if v == 0 else f"val{v}")
        yield workload.terminate_workload(step, total_batches_processed=done), [], workload.ignore_response

    t1 = time.time()
    ctrl = make_controller(model_def.CIFARTrial, cfg, stream(), use_gpu=torch.cuda.is_available(),
                           trial_seed=args.seed)
    t_build = time.time() - t1
    t2 = time.time()
    ctrl.run()
    names = [m[0] for m in marks]
    times = [t2] + [m[1] for m in marks]
    per = {n: times[i + 1] - times[i] for i, n in enumerate(names)}
    trains = [per[n] for n in names if n.startswith("train")]
    steady = trains[1:] if len(trains) > 1 else trains
    steady_batches = args.batches - (args.chunk if len(trains) > 1 else 0)
    ms_batch = 1000.0 * sum(steady) / max(1, steady_batches)
    print(json.dumps({"metric": "CIFAR-10 CNN PyTorchTrial train ms/batch", "value": round(ms_batch, 4),
                      "unit": "ms/batch", "batch": args.batch, "amp": args.amp, "lr": args.lr,
                      "seed": args.seed,
                      "records_per_s": round(args.batch * 1000.0 / ms_batch, 1),
                      "first_chunk_s": round(trains[0], 3), "validation_10k_s": round(per["val"], 3),
                      "validation_10k_s_later": [round(per[n], 4) for n in names if n.startswith("val") and n != "val"],
                      "import_s": round(t_import, 2), "controller_build_s": round(t_build, 2),
                      "hip_graph": ctrl._graph.stats() if getattr(ctrl, "_graph", None) is not None else None,
                      "loss": res[[n for n in names if n.startswith("train")][-1]]["metrics"]["avg_metrics"].get("loss"),
                      "loss_per_chunk": [float(res[n]["metrics"]["avg_metrics"].get("loss", float("nan")))
                                         for n in names if n.startswith("train")],
                      "batch_losses": [float(m["loss"]) for n in names if n.startswith("train")
                                       for m in res[n]["metrics"]["batch_metrics"]] if args.batch_losses else None,
                      "validation_error": float(res["val"]["metrics"]["validation_metrics"].get("validation_error",
                                                                                                float("nan")))},
                     default=float),
          flush=True)


if __name__ == "__main__":
    main()
