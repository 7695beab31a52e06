"""Per-call HBM roofline of the fused BatchNorm kernels in a ResNet-50 training step.

    python scripts/bn_roofline.py [--batch 512] [--iters 5] [--out profiles/r2_bn_bandwidth.csv]

Wraps the det_bn_* entry points of libdetkernels.so (ops/csrc/det_norm.hip) with HIP events, runs
forward+backward of ResNet-50 (bf16 weights and activations, fp32 BN, channels_last, det_conv 1x1
GEMMs: the bench.py O2 configuration), and for every BN call records the bytes it must move
(computed from its shapes and flags) and its GPU time.  A device copy of a 2 GiB buffer measured on
the same box is the achievable-bandwidth reference.  One row per (layer, direction), averaged
over --iters steps, plus totals.
"""
import argparse
import csv
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from determined_1_amd.ops import _lib  # noqa: E402


def copy_bandwidth(dev, nbytes=2 << 30, iters=10) -> float:
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        b.copy_(a)
    e.record()
    torch.cuda.synchronize()
    return 2 * nbytes * iters / (s.elapsed_time(e) * 1e-3) / 1e12


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.get_lib()
    records = []  # (kind, M, C, bytes, ev0, ev1)
    state = {"on": False}

    def wrap(name, nbytes_fn):
        fn = getattr(lib, name)

        def call(*a):
            if not state["on"]:
                return fn(*a)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = fn(*a)
            e1.record()
            kind, m, c, nb = nbytes_fn(a)
            records.append((kind, m, c, nb, e0, e1))
            return rc

        setattr(lib, name, call)

    def fwd_train(a):
        # (stream, dtype, x, res, y, M, C, ..., relu, ..., ws, mbits)
        el = 2 if a[1] == 1 else 4
        m, c = a[5], a[6]
        res, relu, mbits = a[3], a[14], a[20]
        n = m * c * el
        nb = n + n + (n if res else 0) + n + (m * c // 8 if mbits else 0)  # stats read, apply read(+res), write
        return f"fwd{'+res' if res else ''}{'+relu' if relu else ''}", m, c, nb

    def fwd_parts(a):
        # (stream, dtype, x, res, y, M, C, rpb, nrb, pmean, pm2, ..., relu, apply, ..., mbits, ws)
        el = 2 if a[1] == 1 else 4
        m, c, nrb = a[5], a[6], a[8]
        res, relu, apply_, mbits = a[3], a[18], a[19], a[24]
        n = m * c * el
        nb = 2 * nrb * c * 4 + ((n + (n if res else 0) + n + (m * c // 8 if mbits else 0)) if apply_ else 0)
        return f"fwd(gemm-stats){'+res' if res else ''}{'+relu' if relu else ''}", m, c, nb

    def bwd(a):
        # (stream, dtype, dy, dy2, x, mbits, M, C, mask_mode, ..., dx, dres, dgamma, dbeta, ws)
        el = 2 if a[1] == 1 else 4
        dy2, mbits, m, c, mode, dres = a[3], a[5], a[6], a[7], a[8], a[15]
        n = m * c * el
        mb = m * c // 8 if (mode == 2 and mbits) else 0
        part = n + (n if dy2 else 0) + n + mb
        apply_ = n + (n if dy2 else 0) + n + mb + n + (n if dres else 0)
        return f"bwd{'+dy2' if dy2 else ''}{'+dres' if dres else ''} mask{mode}", m, c, part + apply_

    wrap("det_bn_fwd_train", fwd_train)
    wrap("det_bn_fwd_from_partials", fwd_parts)
    wrap("det_bn_bwd", bwd)

    from determined_1_amd.models import resnet

    torch.manual_seed(0)
    model = resnet.resnet50(num_classes=1000).to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16)
    for mod in model.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.float()
    x = torch.randn(args.batch, 3, args.image_size, args.image_size, device=dev).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.batch,), device=dev)

    def step():
        model.zero_grad(set_to_none=True)
        loss = torch.nn.functional.cross_entropy(model(x).float(), y)
        loss.backward()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    state["on"] = True
    for _ in range(args.iters):
        step()
    torch.cuda.synchronize()
    state["on"] = False
    copy_tbs = copy_bandwidth(dev)

    per_step = len(records) // args.iters
    rows = []
    for i in range(per_step):
        group = [records[i + k * per_step] for k in range(args.iters)]
        kind, m, c, nb = group[0][:4]
        ms = sum(g[4].elapsed_time(g[5]) for g in group) / len(group)
        tbs = nb / (ms * 1e-3) / 1e12
        rows.append((i, kind, m, c, nb, ms, tbs, 100.0 * tbs / copy_tbs))
    tot_b = sum(r[4] for r in rows)
    tot_ms = sum(r[5] for r in rows)
    print(f"device copy bandwidth: {copy_tbs:.2f} TB/s (read+write of a 2 GiB buffer)")
    print(f"{'#':>3} {'call':<34} {'M':>9} {'C':>5} {'MB':>9} {'ms':>7} {'TB/s':>6} {'%copy':>6}")
    for r in rows:
        print(f"{r[0]:>3} {r[1]:<34} {r[2]:>9} {r[3]:>5} {r[4] / 1e6:>9.1f} {r[5]:>7.3f} {r[6]:>6.2f} {r[7]:>6.1f}")
    print(f"TOTAL {len(rows)} BN calls/step: {tot_b / 1e9:.2f} GB, {tot_ms:.3f} ms, {tot_b / (tot_ms * 1e-3) / 1e12:.2f} TB/s "
          f"({100.0 * tot_b / (tot_ms * 1e-3) / 1e12 / copy_tbs:.1f}% of copy)")
    if args.out:
        with open(args.out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["idx", "call", "M", "C", "bytes", "ms", "TB_s", "pct_of_copy_bw"])
            w.writerow(["copy", f"device copy 2GiB (batch {args.batch})", "", "", "", "", f"{copy_tbs:.3f}", "100.0"])
            for r in rows:
                w.writerow([r[0], r[1], r[2], r[3], r[4], f"{r[5]:.4f}", f"{r[6]:.3f}", f"{r[7]:.1f}"])
            w.writerow(["total", f"{len(rows)} calls", "", "", tot_b, f"{tot_ms:.4f}",
                        f"{tot_b / (tot_ms * 1e-3) / 1e12:.3f}", f"{100.0 * tot_b / (tot_ms * 1e-3) / 1e12 / copy_tbs:.1f}"])


if __name__ == "__main__":
    main()
