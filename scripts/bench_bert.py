"""BERT-base SQuAD-shape throughput through the real PyTorchTrial path (BASELINE config 5 shape:
seq 384, per-GPU batch 12 (global 96 on 8 GPUs), AdamW fused HIP kernel, bf16 AMP O2, clipping).

    python scripts/bench_bert.py [--steps K] [--warmup W] [--batch-per-gpu B] [--amp O2]
One JSON line: examples/s (whole node) + ms/step.  Multi-GPU: launch with torch.distributed.run.
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch-per-gpu", type=int, default=12)
    ap.add_argument("--amp", default="O2")
    ap.add_argument("--agg", type=int, default=1, help="optimizations.aggregation_frequency")
    ap.add_argument("--impl", default="native", choices=["native", "hf"], help="fused MI355X encoder or HF BERT")
    ap.add_argument("--hip-graph", action="store_true", help="optimizations.hip_graph: replay train_batch as a hipGraph")
    ap.add_argument("--no-dropout", action="store_true", help="dropout 0 (graph vs eager parameter comparisons)")
    ap.add_argument("--params-out", default="", help="save per-tensor float64 sums / norms of the final parameters")
    ap.add_argument("--loss-every", type=int, default=0,
                    help="timed steps in workloads of this many batches, reporting each one's mean loss (long-run "
                         "graph-vs-eager tracking)")
    ap.add_argument("--cprof", default="", help="write a cProfile of the timed steps to this path")
    ap.add_argument("--autograd-threads", type=int, default=0,
                    help="1: stock multithreaded autograd engine (the controller disables it by default)")
    args = ap.parse_args()
    if os.environ.get("DET_STEP_TIMERS"):
        import logging

        logging.basicConfig(level=logging.INFO, format="%(message)s")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    from determined_1_amd.parallel import dist as pdist

    if torch.cuda.is_available():
        torch.cuda.set_device(pdist.local_cuda_device(int(os.environ.get("LOCAL_RANK", "0"))))
    from determined_1_amd import workload
    from determined_1_amd.experimental import make_controller
    from determined_1_amd.experimental import load_model_def

    BertSQuADTrial = load_model_def(os.path.join(REPO, "examples", "nlp", "bert_squad_pytorch")).BertSQuADTrial
    from determined_1_amd.parallel import dist as pdist

    gbs = args.batch_per_gpu * world
    cfg = {
        "hyperparameters": {"global_batch_size": gbs, "learning_rate": 3e-5, "max_seq_length": 384, "amp": args.amp,
                            "max_grad_norm": 1.0, "train_records": 100000, "impl": args.impl,
                            **({"hidden_dropout_prob": 0.0, "attention_probs_dropout_prob": 0.0} if args.no_dropout else {})},
        "resources": {"slots_per_trial": world},
        "optimizations": {"aggregation_frequency": args.agg, "hip_graph": bool(args.hip_graph)},
        "searcher": {"name": "single", "metric": "f1", "max_length": {"batches": args.steps}, "smaller_is_better": False},
    }
    t = {}

    def sync() -> None:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        pdist.barrier()

    prof = None
    if args.cprof:
        import cProfile

        prof = cProfile.Profile()
    if args.autograd_threads:
        os.environ["DET_AUTOGRAD_THREADS"] = "1"

    losses = []

    def keep_loss(r) -> None:
        m = (r or {}).get("metrics", {}).get("avg_metrics", {}) if isinstance(r, dict) else {}
        if "loss" in m:
            losses.append(float(m["loss"]))
            print(f"[bench_bert] {len(losses) * args.loss_every} steps, loss {losses[-1]:.5f}, "
                  f"{time.perf_counter() - t['t0']:.1f}s", file=sys.stderr, flush=True)

    def stream():
        yield workload.train_workload(1, num_batches=args.warmup), [], workload.ignore_response
        sync()
        if prof is not None:
            prof.enable()
        t["t0"] = time.perf_counter()
        if args.loss_every > 0:
            done, step = 0, 2
            while done < args.steps:
                n = min(args.loss_every, args.steps - done)
                yield (workload.train_workload(step, num_batches=n, total_batches_processed=args.warmup + done), [],
                       keep_loss)
                done += n
                step += 1
        else:
            yield (workload.train_workload(2, num_batches=args.steps, total_batches_processed=args.warmup), [],
                   workload.ignore_response)
        sync()
        t["t1"] = time.perf_counter()
        if prof is not None:
            prof.disable()
            prof.dump_stats(args.cprof)
        yield workload.terminate_workload(10 ** 6), [], workload.ignore_response

    ctrl = make_controller(BertSQuADTrial, cfg, stream(), trial_seed=7)
    ctrl.run()
    g = getattr(ctrl, "_graph", None)
    graph_stats = {k: getattr(g, k, None) for k in ("captures", "failed_captures", "replays")} if g is not None else None
    el = max(pdist.allgather_object(t["t1"] - t["t0"]))
    if args.params_out and rank == 0:
        ps = [p.detach().double() for p in ctrl.context.models[0].parameters()]
        torch.save({"sums": torch.stack([p.sum() for p in ps]).cpu(), "norms": torch.stack([p.norm() for p in ps]).cpu(),
                    "head": torch.cat([p.reshape(-1)[:64] for p in ps]).cpu()}, args.params_out)
    from determined_1_amd.ops import transformer as tfops

    if rank == 0:
        print(json.dumps({"metric": "examples/sec (whole node) BERT-base SQuAD-shape PyTorchTrial",
                          "value": round(args.steps * gbs / el, 2), "unit": "examples/s", "n_gpus": world,
                          "ms_per_step": round(1000 * el / args.steps, 2), "dtype": "bf16" if args.amp != "O0" else "fp32",
                          "config": {"model": "bert-base (random init)", "seq_len": 384, "global_batch": gbs,
                                     "amp": args.amp, "aggregation_frequency": args.agg,
                                     "optimizer": "AdamW (fused arena HIP kernel)", "impl": args.impl,
                                     "hip_graph": bool(args.hip_graph), "graph_stats": graph_stats,
                                     "tf_fallbacks": tfops.FALLBACKS["count"]},
                          "losses": [round(x, 5) for x in losses] if losses else None}), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
