"""Detection training throughput through the real PyTorchTrial path, at the reference configs:

  --model detr        ``detr_coco_pytorch/const_fake.yaml``: DETR-R50 (6+6 layers, 100 queries),
                      per-GPU batch 2, AdamW (backbone lr 1e-5), clip 0.1, aux losses; synthetic
                      COCO-shaped images (the reference's ``fake`` backend) of 480-640 px, padded
                      per batch.  A step = forward, Hungarian matching of all 6 decoder layers,
                      backward, clip, AdamW.
  --model maskrcnn    ``maskrcnn_coco_pytorch/const.yaml`` (stands in for the reference's
                      mmdetection ``maskrcnn.yaml``; it publishes 0.310 s/iter at 2 images per V100):
                      Mask R-CNN R50-FPN, 2 images per GPU, SGD, COCO-shaped 480-640 px synthetic
                      instances resized to 800 px short side.
  --model fasterrcnn  ``fasterrcnn_coco_pytorch/const.yaml``: Faster R-CNN R50-FPN, batch 2, SGD
                      momentum; PennFudan-sized synthetic images (300-500 px) resized to 800 px
                      short side as torchvision's transform does.  A step = full detector forward
                      (RPN + RoI heads losses) and backward of ``loss_box_reg`` (what the reference
                      trains on), SGD.

    python scripts/bench_detection.py --model detr|fasterrcnn [--steps K] [--warmup W]
        [--batch-per-gpu B] [--amp O0|O2] [--min-size N --max-size N]

The reference publishes no throughput for either example.
"""
import argparse
import importlib.util
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# the shipped MIOpen find-db / kernel cache (seeded for the bucketed detection shapes by
# scripts/miopen_seed_detection.py), configured before torch initialises MIOpen
_spec = importlib.util.spec_from_file_location("_det_miopen_db", os.path.join(REPO, "determined_1_amd", "ops", "miopen_db.py"))
_mdb = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(_mdb)  # type: ignore
_mdb.configure(os.environ)

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-per-gpu", type=int, default=2)
    ap.add_argument("--amp", default="O0", help="O0 = fp32 as the reference config; O2 = bf16 weights + fp32 master")
    ap.add_argument("--model", choices=["detr", "fasterrcnn", "maskrcnn", "retinanet"], default="detr")
    ap.add_argument("--min-size", type=int, default=0, help="synthetic image side range (0: model default)")
    ap.add_argument("--max-size", type=int, default=0)
    ap.add_argument("--small", action="store_true", help="tiny model (CPU smoke only)")
    ap.add_argument("--coco-instances", action="store_true",
                    help="COCO-like instance load (mean 7.3 per image, heavy tail, small objects) for Mask R-CNN / RetinaNet")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    from determined_1_amd.parallel import dist as pdist

    if torch.cuda.is_available():
        torch.cuda.set_device(pdist.local_cuda_device(int(os.environ.get("LOCAL_RANK", "0"))))
    from determined_1_amd import workload
    from determined_1_amd.experimental import load_model_def, make_controller

    import yaml

    if args.model == "detr":
        ex = os.path.join(REPO, "examples", "computer_vision", "detr_coco_pytorch")
        Trial = load_model_def(ex).DETRTrial
        cfg = yaml.safe_load(open(os.path.join(ex, "const_fake.yaml")))
        lo, hi = args.min_size or 480, args.max_size or 640
        metric, model_name = "mAP", "detr-r50 6enc/6dec/100q"
    elif args.model == "retinanet":
        ex = os.path.join(REPO, "examples", "computer_vision", "retinanet_coco_pytorch")
        Trial = load_model_def(ex).RetinaNetTrial
        cfg = yaml.safe_load(open(os.path.join(ex, "const.yaml")))
        lo, hi = args.min_size or 480, args.max_size or 640
        metric, model_name = "val_box_iou", "retinanet-r50-fpn 800px (mmdet retinanet_r50_fpn_1x shape)"
    elif args.model == "maskrcnn":
        ex = os.path.join(REPO, "examples", "computer_vision", "maskrcnn_coco_pytorch")
        Trial = load_model_def(ex).MaskRCNNTrial
        cfg = yaml.safe_load(open(os.path.join(ex, "const.yaml")))
        lo, hi = args.min_size or 480, args.max_size or 640
        metric, model_name = "val_mask_iou", "maskrcnn-r50-fpn 800px (mmdet mask_rcnn_r50_fpn_1x shape)"
    else:
        ex = os.path.join(REPO, "examples", "computer_vision", "fasterrcnn_coco_pytorch")
        Trial = load_model_def(ex).ObjectDetectionTrial
        cfg = yaml.safe_load(open(os.path.join(ex, "const.yaml")))
        lo, hi = args.min_size or 300, args.max_size or 500
        metric, model_name = "val_avg_iou", "fasterrcnn-r50-fpn 800px"
    hp = dict(cfg["hyperparameters"])
    gbs = args.batch_per_gpu * world
    hp.update(global_batch_size=gbs, amp=args.amp, min_image_size=lo, max_image_size=hi, num_workers=2)
    if args.model == "fasterrcnn":
        hp["num_images"] = max(int(hp.get("num_images", 170)), (args.steps + args.warmup) * gbs * 2)
    if args.model in ("maskrcnn", "retinanet"):
        hp["train_records"] = max(int(hp.get("train_records", 2000)), (args.steps + args.warmup) * gbs)
        if args.coco_instances:
            hp["instance_dist"] = "coco"
            model_name += ", COCO-like instance load"
    if args.small:
        hp.update(backbone="resnet26", enc_layers=1, dec_layers=2, hidden_dim=32, nheads=2, dim_feedforward=64,
                  num_queries=10, num_workers=0, transform_min_size=96, transform_max_size=160)
        model_name += " (small smoke)"
    steps, warm = args.steps, args.warmup
    cfg = {"hyperparameters": hp, "resources": {"slots_per_trial": world}, "records_per_epoch": 117264,
           "searcher": {"name": "single", "metric": metric, "max_length": {"batches": steps + warm},
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
            print(f"[bench_detection rank{rank}] {'timed' if 't0' in t else 'warmup'} {time.perf_counter() - t_start:.0f}s",
                  file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    ctrl = make_controller(Trial, cfg, stream(), trial_seed=7)
    ctrl.run()
    el = max(pdist.allgather_object(t["t1"] - t["t0"]))
    from determined_1_amd.ops import conv as _native_conv

    if rank == 0:
        print(json.dumps({
            "metric": f"images/sec (whole node) {args.model} PyTorchTrial", "value": round(steps * gbs / el, 2),
            "unit": "images/s", "n_gpus": world, "steps": steps, "warmup": warm,
            "ms_per_step": round(1000 * el / steps, 2), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16" if args.amp != "O0" else "fp32",
            "data": f"synthetic detection images {lo}-{hi}px; random-init weights",
            "config": {"model": model_name, "per_gpu_batch": args.batch_per_gpu, "global_batch": gbs, "amp": args.amp,
                       "optimizer": "AdamW, backbone lr 1e-5, clip 0.1" if args.model == "detr" else "SGD momentum",
                       "s_per_iter": round(el / steps, 4),
                       "native_conv2d": dict(_native_conv.CONV2D_COUNTS), "native_conv2d_on": _native_conv.NATIVE_CONV2D,
                       "parallelism": f"dp{world}"}}), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
