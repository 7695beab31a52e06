"""Harness overhead check ("harness overhead target <= 2 % vs a bare PyTorch loop at
the same config"): the ResNet-50 step of ``bench.py`` written as a bare loop — same model, same
fused BN / pool HIP kernels, same u8 -> bf16 input kernel, same bf16 O2 weights, same fused arena
SGD kernel with gradient landing — but no ``PyTorchTrialController``, no workload stream, no
DataLoader/prefetcher (one resident synthetic batch), no metric collection.  ``bench.py`` minus
this = what the harness costs.

    python scripts/bench_bare.py --steps 30 --warmup 10 [--batch-per-gpu 512]

Prints one JSON line (1 GPU).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-per-gpu", type=int, default=512)
    ap.add_argument("--image-size", type=int, default=224)
    args = ap.parse_args()

    from determined_1_amd.models import resnet
    from determined_1_amd.models.synthetic import IMAGENET_MEAN, IMAGENET_STD
    from determined_1_amd.ops.arena import GradSink
    from determined_1_amd.ops.functional import u8_normalize
    from determined_1_amd.ops.optim import FusedOptimizer

    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    resnet.FUSED_BN = True
    model = resnet.resnet50(num_classes=1000).to(dev).to(memory_format=torch.channels_last)
    # O2: bf16 weights except BatchNorm; the fused optimizer keeps fp32 masters in its arena
    for m in model.modules():
        if not isinstance(m, nn.modules.batchnorm._BatchNorm):
            for p in m.parameters(recurse=False):
                p.data = p.data.to(torch.bfloat16)
    opt = torch.optim.SGD(model.parameters(), lr=0.1 * args.batch_per_gpu / 256, momentum=0.9, weight_decay=5e-5)
    fused = FusedOptimizer(opt, dev)
    fused.sink = GradSink.for_arenas(fused.arenas)
    loss_fn = nn.CrossEntropyLoss()
    bs, hw = args.batch_per_gpu, args.image_size
    images = torch.randint(0, 256, (bs, hw, hw, 3), dtype=torch.uint8, device=dev)
    labels = torch.randint(0, 1000, (bs,), device=dev)

    def step() -> torch.Tensor:
        x = u8_normalize(images, IMAGENET_MEAN, IMAGENET_STD, out_dtype=torch.bfloat16)
        loss = loss_fn(model(x).float(), labels)
        loss.backward()
        opt.step()
        opt.zero_grad()
        return loss

    opt.zero_grad()
    t_start = time.perf_counter()
    for i in range(args.warmup):
        step()
        torch.cuda.synchronize()
        print(f"[bare] warmup {i} {time.perf_counter() - t_start:.0f}s", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    print(json.dumps({"metric": "samples/sec bare loop ResNet-50 (no harness)", "value": round(args.steps * bs / t, 2),
                      "unit": "samples/s", "ms_per_step": round(1000 * t / args.steps, 3), "steps": args.steps,
                      "warmup": args.warmup, "per_gpu_batch": bs, "final_loss": float(loss)}), flush=True)


if __name__ == "__main__":
    main()
