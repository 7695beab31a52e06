"""ALBERT-xxlarge-v2 SQuAD-shape fine-tuning throughput through the real PyTorchTrial path — the
workload behind the reference's only published throughput numbers
(``examples/nlp/albert_squad_pytorch/README.md:25-29``: 2 examples/s on 1 V100-16GB, 15.8 on 8,
92.75 on 64; configs ``const.yaml`` / ``distributed_8gpu.yaml``: seq 384, AdamW, clipping 1.0,
per-GPU batch 2 with aggregation_frequency 24 (1 GPU) / 3 (8 GPUs) = 48 examples per update).

    python scripts/bench_albert.py [--steps K] [--warmup W] [--batch-per-gpu B] [--agg A]
    python -m torch.distributed.run --nproc-per-node N scripts/bench_albert.py ...

The 288 GB of an MI355X hold a larger per-GPU batch than a 16 GB V100, so the default is 8 per
GPU with aggregation_frequency chosen to keep >= 48 examples per optimizer update (6 on one GPU,
1 on eight).  A "step" is one batch (the reference's throughput counts examples, not updates).
Weights are random-init albert-xxlarge-v2 geometry, data is synthetic SQuAD-shaped features.
"""
import argparse
import json
import os
import sys
import threading
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

PUBLISHED = {1: 2.0, 8: 15.8, 64: 92.75}  # examples/s, V100-16GB (README.md:27-29)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--batch-per-gpu", type=int, default=8)
    ap.add_argument("--agg", type=int, default=0, help="aggregation_frequency (0: keep >= 48 examples per update)")
    ap.add_argument("--amp", default="O2")
    ap.add_argument("--layers", type=int, default=12, help="(smoke tests only; the metric is 12)")
    ap.add_argument("--hidden", type=int, default=4096, help="(smoke tests only; the metric is 4096)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    from determined_1_amd.parallel import dist as pdist

    if torch.cuda.is_available():
        torch.cuda.set_device(pdist.local_cuda_device(int(os.environ.get("LOCAL_RANK", "0"))))
    from determined_1_amd import workload
    from determined_1_amd.experimental import make_controller
    from determined_1_amd.experimental import load_model_def

    AlbertSQuADTrial = load_model_def(os.path.join(REPO, "examples", "nlp", "albert_squad_pytorch")).AlbertSQuADTrial
    from determined_1_amd.ops import transformer as tfops
    from determined_1_amd.parallel import dist as pdist

    gbs = args.batch_per_gpu * world
    agg = args.agg or max(1, -(-48 // gbs))
    steps = -(-args.steps // agg) * agg  # whole aggregation windows in the timed region
    warm = -(-args.warmup // agg) * agg
    hp = {"global_batch_size": gbs, "learning_rate": 5e-5, "max_seq_length": 384, "amp": args.amp,
          "max_grad_norm": 1.0, "weight_decay": 0.0, "adam_epsilon": 1e-8, "num_warmup_steps": 1620,
          "num_training_steps": 16500, "train_records": 132198}
    if args.layers != 12 or args.hidden != 4096:
        hp.update(num_hidden_layers=args.layers, hidden_size=args.hidden, intermediate_size=4 * args.hidden,
                  num_attention_heads=max(1, args.hidden // 64))
    cfg = {"hyperparameters": hp, "resources": {"slots_per_trial": world},
           "optimizations": {"aggregation_frequency": agg},
           "searcher": {"name": "single", "metric": "f1", "max_length": {"batches": steps}, "smaller_is_better": False}}
    t = {}

    def sync() -> None:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        pdist.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def stream():
        yield workload.train_workload(1, num_batches=warm), [], workload.ignore_response
        sync()
        t["t0"] = time.perf_counter()
        yield workload.train_workload(2, num_batches=steps, total_batches_processed=warm), [], workload.ignore_response
        sync()
        t["t1"] = time.perf_counter()
        yield workload.terminate_workload(3), [], workload.ignore_response

    t_start = time.perf_counter()

    def heartbeat() -> None:
        while True:
            time.sleep(30)
            print(f"[bench_albert rank{rank}] {'timed' if 't0' in t else 'warmup'} {time.perf_counter() - t_start:.0f}s",
                  file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    ctrl = make_controller(AlbertSQuADTrial, cfg, stream(), trial_seed=11)
    ctrl.run()
    el = max(pdist.allgather_object(t["t1"] - t["t0"]))
    value = steps * gbs / el
    if rank == 0:
        base = PUBLISHED.get(world)
        print(json.dumps({
            "metric": "examples/sec (whole node) ALBERT-xxlarge-v2 SQuAD-shape PyTorchTrial",
            "value": round(value, 2), "unit": "examples/s", "n_gpus": world, "steps": steps, "warmup": warm,
            "ms_per_step": round(1000 * el / steps, 2), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / base, 2) if base and args.layers == 12 and args.hidden == 4096 else None,
            "baseline": f"{base} examples/s on {world}x V100-16GB (albert_squad_pytorch/README.md)" if base else None,
            "dtype": "bf16" if args.amp != "O0" else "fp32", "data": "synthetic SQuAD-shaped features; random-init weights",
            "config": {"model": "albert-xxlarge-v2" if args.layers == 12 and args.hidden == 4096 else
                       f"albert {args.layers}x{args.hidden} (smoke)", "seq_len": 384, "per_gpu_batch": args.batch_per_gpu,
                       "global_batch": gbs, "aggregation_frequency": agg, "amp": args.amp,
                       "optimizer": "AdamW (fused arena HIP kernel) + clip 1.0", "parallelism": f"dp{world}",
                       "tf_fallbacks": tfops.FALLBACKS["count"]}}), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
