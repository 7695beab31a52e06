"""DETR (ResNet-50, 6+6 layers, 100 queries) training throughput through the real PyTorchTrial
path at the reference ``detr_coco_pytorch/const_fake.yaml`` config: per-GPU batch 2, AdamW with
backbone lr 1e-5, clip 0.1, aux losses; synthetic COCO-shaped images (the reference's ``fake``
backend) of 480-640 px per side, padded per batch.  The reference publishes no DETR throughput.

    python scripts/bench_detr.py [--steps K] [--warmup W] [--batch-per-gpu B] [--amp O0|O2]
                                 [--min-size 480 --max-size 640]

A step = one batch (forward, Hungarian matching of all 6 decoder layers, backward, clip, AdamW).
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


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-per-gpu", type=int, default=2)
    ap.add_argument("--amp", default="O0", help="O0 = fp32 as the reference config; O2 = bf16 weights + fp32 master")
    ap.add_argument("--min-size", type=int, default=480)
    ap.add_argument("--max-size", type=int, default=640)
    ap.add_argument("--small", action="store_true", help="tiny model (CPU smoke only)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    from determined_1_amd.parallel import dist as pdist

    if torch.cuda.is_available():
        torch.cuda.set_device(pdist.local_cuda_device(int(os.environ.get("LOCAL_RANK", "0"))))
    from determined_1_amd import workload
    from determined_1_amd.experimental import load_model_def, make_controller

    DETRTrial = load_model_def(os.path.join(REPO, "examples", "computer_vision", "detr_coco_pytorch")).DETRTrial
    import yaml

    cfg = yaml.safe_load(open(os.path.join(REPO, "examples", "computer_vision", "detr_coco_pytorch", "const_fake.yaml")))
    hp = dict(cfg["hyperparameters"])
    gbs = args.batch_per_gpu * world
    hp.update(global_batch_size=gbs, amp=args.amp, min_image_size=args.min_size, max_image_size=args.max_size,
              num_workers=2)
    if args.small:
        hp.update(backbone="resnet26", enc_layers=1, dec_layers=2, hidden_dim=32, nheads=2, dim_feedforward=64,
                  num_queries=10, num_workers=0)
    steps, warm = args.steps, args.warmup
    cfg = {"hyperparameters": hp, "resources": {"slots_per_trial": world}, "records_per_epoch": 117264,
           "searcher": {"name": "single", "metric": "mAP", "max_length": {"batches": steps + warm},
                        "smaller_is_better": False}}
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
            time.sleep(20)
            print(f"[bench_detr rank{rank}] {'timed' if 't0' in t else 'warmup'} {time.perf_counter() - t_start:.0f}s",
                  file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    ctrl = make_controller(DETRTrial, cfg, stream(), trial_seed=7)
    ctrl.run()
    el = max(pdist.allgather_object(t["t1"] - t["t0"]))
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec (whole node) DETR-R50 COCO-shape PyTorchTrial", "value": round(steps * gbs / el, 2),
            "unit": "images/s", "n_gpus": world, "steps": steps, "warmup": warm,
            "ms_per_step": round(1000 * el / steps, 2), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16" if args.amp != "O0" else "fp32",
            "data": f"synthetic COCO-shaped images {args.min_size}-{args.max_size}px with 1-6 boxes; random-init weights",
            "config": {"model": "detr-r50 (small smoke)" if args.small else "detr-r50 6enc/6dec/100q", "per_gpu_batch":
                       args.batch_per_gpu, "global_batch": gbs, "amp": args.amp,
                       "optimizer": "AdamW (fused arena HIP kernel), backbone lr 1e-5, clip 0.1",
                       "parallelism": f"dp{world}"}}), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
