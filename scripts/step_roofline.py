"""Per-call roofline of every native kernel in a ResNet-50 training step ("a byte model
whose rows are all <= 100 % of measured copy bandwidth").

    python scripts/step_roofline.py [--batch 512] [--iters 3] [--out profiles/r4_step_roofline.csv]

Wraps the det_* entry points of libdetkernels.so with HIP events, runs forward + backward of the
benchmark's ResNet-50 (bf16 channels_last, fused BN, native convs), and for every call records its
compulsory HBM bytes (each tensor argument read or written once -- re-reads that a kernel serves from
L2 / the 256 MiB Infinity Cache are not counted) and its FLOPs.  The bandwidth reference of each row
is a device copy of the SAME number of bytes measured on the same box (half read, half written), so
an L3-resident small tensor is held to an L3-speed copy, not to the HBM rate: rows above 100 % then
mean the byte model is wrong.  Prints one row per call and a summary per kernel family."""
import argparse
import csv
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from determined_1_amd.ops import _lib  # noqa: E402

_COPY = {}


def copy_tbs(dev, nbytes: int) -> float:
    """Throughput of a device copy moving ``nbytes`` in total (nbytes/2 read + nbytes/2 written),
    freshly written source (as a producer kernel leaves it)."""
    key = max(1 << 20, 1 << int(nbytes).bit_length())  # power-of-two buckets
    if key not in _COPY:
        n = key // 4
        a = torch.empty(n // 2, dtype=torch.float32, device=dev)
        b = torch.empty_like(a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t = 0.0
        for _ in range(5):
            a.fill_(1.0)
            e0.record()
            b.copy_(a)
            e1.record()
            torch.cuda.synchronize()
            t += e0.elapsed_time(e1)
        _COPY[key] = key / (t / 5 * 1e-3) / 1e12
    return _COPY[key]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.get_lib()
    recs = []
    state = {"on": False}

    def wrap(name, model):
        fn = getattr(lib, name)

        def call(*a):
            if not state["on"]:
                return fn(*a)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = fn(*a)
            e1.record()
            kind, nbytes, flops = model(a)
            recs.append((name, kind, nbytes, flops, e0, e1))
            return rc

        setattr(lib, name, call)

    el = lambda dt: 2 if dt == 1 else 4  # noqa: E731

    # ---- BatchNorm family (det_norm.hip)
    def bn_fwd_train(a):
        m, c, n = a[5], a[6], a[5] * a[6] * el(a[1])
        return ("bn fwd (stats+apply)", 2 * n + (n if a[3] else 0) + (m * c // 8 if a[20] else 0), 0)

    def bn_stats(a):
        return ("bn stats", a[3] * a[4] * el(a[1]), 0)

    def bn_fwd_parts(a):
        m, c, nrb, n = a[5], a[6], a[8], a[5] * a[6] * el(a[1])
        apply_ = a[19]
        b = 2 * nrb * c * 4 + ((2 * n + (n if a[3] else 0) + (m * c // 8 if a[24] else 0)) if apply_ else 0)
        return ("bn fwd finalize" + (" + apply" if apply_ else ""), b, 0)

    def bn_apply(a):
        n = a[5] * a[6] * el(a[1])
        return ("bn apply (frozen)", 2 * n + (n if a[3] else 0), 0)

    def bn_apply_res_mbits(a):
        m, c = a[4], a[5]
        return ("bn apply + res + mask (deferred)", 3 * m * c * 2 + m * c // 8, 0)

    def bn_bwd(a):
        m, c, mode, n = a[6], a[7], a[8], a[6] * a[7] * el(a[1])
        b = n + (n if a[3] else 0) + n + (m * c // 8 if mode == 2 and a[5] else 0) + n + (n if a[15] else 0)
        return (f"bn bwd (partials+apply) mask{mode}", b, 0)

    def bn_bwd_parts(a):
        m, c, nrb, n = a[4], a[5], a[11], a[4] * a[5] * el(a[1])
        return ("bn bwd finalize + apply", 3 * n + 2 * nrb * c * 4, 0)

    def bn_bwd_fin(a):
        return ("bn bwd finalize", 2 * a[8] * a[2] * 4, 0)  # (nrb, rpb) = a[8], a[9]

    def bn_bwd_coef(a):
        n = a[4] * a[5] * el(a[1])
        return ("bn bwd apply (materialised)", 3 * n, 0)

    # ---- convolutions (det_conv.hip / det_igemm.hip)
    def conv_nt(a):
        m, n, k = a[4], a[5], a[6]
        gather = a[11] > 0
        b = m * k * 2 + n * k * 2 + m * n * 2
        kind = "1x1 fwd" + (" s2" if gather else "") + (" +stats" if a[9] else "") + (" +prologue" if a[7] else "")
        if a[15]:  # AFWD: also reads the residual, writes the applied A and its mask bits (first N tile)
            b += m * k * 2 + m * k * 2 + m * k // 8
            kind = "1x1 fwd + bn3 apply (AFWD)"
        return (kind, b, 2 * m * n * k)

    def conv_dgrad(a):
        m, n, k = a[4], a[5], a[6]
        b = m * k * 2 + n * k * 2 + m * n * 2 + (2 * m * k * 2 if a[7] else 0)
        return ("1x1 dgrad" + (" + bn bwd apply (ABN)" if a[7] else ""), b, 2 * m * n * k)

    def conv_nt_bnbwd(a):
        m, n, k, mode = a[4], a[5], a[6], a[15]
        b = m * k * 2 + n * k * 2 + 2 * m * n * 2  # dY, W, write d, read bn x
        if a[12]:
            sub = a[20] > 0
            b += (m * n * 2 // 4 if sub else m * n * 2)  # shortcut gradient (stride-2 grid: a quarter)
        if mode == 2:
            b += m * n // 8
        if a[17]:
            b += 2 * m * k * 2
        return (f"1x1 dgrad + bn bwd epilogue mask{mode}" + (" + ABN" if a[17] else ""), b, 2 * m * n * k)

    def conv_tn(a):
        m, n, k = a[5], a[6], a[7]
        return ("1x1 wgrad (gemm_tn)", m * n * 2 + m * k * 2 + n * k * 4, 2 * m * n * k)

    def conv_wgrad(a):
        m, n, cin, r, s = a[5], a[6], a[7], a[12], a[13]
        hi, wi, ho, wo = a[8], a[9], a[10], a[11]
        x = (m // (ho * wo)) * hi * wi * cin * 2
        return (f"{r}x{s} wgrad (gemm_tn im2col)", m * n * 2 + x + n * r * s * cin * 4, 2 * m * n * r * s * cin)

    def igemm_wgrad(a):
        m, n, cin, r, s = a[5], a[6], a[7], a[12], a[13]
        hi, wi, ho, wo = a[8], a[9], a[10], a[11]
        x = (m // (ho * wo)) * hi * wi * cin * 2
        return (f"{r}x{s} wgrad (ring)", m * n * 2 + x + n * r * s * cin * 4, 2 * m * n * r * s * cin)

    def igemm_conv(a):
        m, n, cin, hi, wi, ho, wo, r, s = a[5], a[6], a[7], a[8], a[9], a[10], a[11], a[12], a[13]
        x = (m // (ho * wo)) * hi * wi * cin * 2
        kind = f"{r}x{s} s{a[14]} igemm" + (" +stats" if a[16] else "")
        return (kind, x + n * r * s * cin * 2 + m * n * 2, 2 * m * n * r * s * cin)

    def igemm_bnbwd(a):
        m, n, cin, hi, wi, ho, wo, r, s = a[5], a[6], a[7], a[8], a[9], a[10], a[11], a[12], a[13]
        x = (m // (ho * wo)) * hi * wi * cin * 2
        return (f"{r}x{s} dgrad igemm + bn bwd epilogue", x + n * r * s * cin * 2 + 2 * m * n * 2, 2 * m * n * r * s * cin)

    def dgrad_s2(a):
        nb, ho, wo, cout, cin = a[5], a[6], a[7], a[8], a[9]
        m_in = nb * 4 * ho * wo
        b = nb * ho * wo * cout * 2 + 9 * cin * cout * 2 + m_in * cin * 2 + (m_in * cin * 2 if a[10] else 0)
        return ("3x3 s2 dgrad (parity classes)" + (" + bn bwd epilogue" if a[10] else ""), b, 2 * m_in * cin * cout * 9 // 4)

    def conv3p(a):
        nb, h, w, cin, n = a[4], a[5], a[6], a[7], a[8]
        m = nb * h * w
        b = m * cin * 2 + 9 * n * cin * 2 + m * n * 2 + (m * n * 2 if a[13] else 0)
        kind = "3x3 conv3p" + (" dgrad + bn bwd epilogue" if a[13] else (" +stats" if a[11] else ""))
        return (kind, b, 2 * m * n * 9 * cin)

    def conv3p_wgrad(a):
        nb, h, w, cin, n = a[5], a[6], a[7], a[8], a[9]
        m = nb * h * w
        return ("3x3 wgrad (conv3p patch)", m * n * 2 + m * cin * 2 + 9 * n * cin * 4, 2 * m * n * 9 * cin)

    def stem_fwd(a):
        m, hi, wi = a[4], a[5], a[6]
        nimg = m // (a[7] * a[8])
        return ("stem 7x7 fwd +stats", nimg * hi * wi * 8 + m * 64 * 2, 2 * m * 64 * 147)

    def stemp(a):
        m, hi, wi, ho, wo = a[5], a[6], a[7], a[8], a[9]
        return ("stem wgrad (patch)", m * 128 + (m // (ho * wo)) * hi * wi * 8, 2 * m * 64 * 147)

    def dgrad_weight(a):
        k, c, r, s = a[4], a[5], a[6], a[7]
        return ("dgrad weight flip", k * c * r * s * (2 if a[2] == 1 else 4) + k * c * r * s * 2, 0)

    def maxpool_fwd(a):
        n, h, w, c = a[5], a[6], a[7], a[8]
        ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        return ("maxpool fwd", n * h * w * c * 2 + n * ho * wo * c * 3, 0)

    def maxpool_bwd(a):
        n, h, w, c = a[6], a[7], a[8], a[9]
        ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        linked = n * ho * wo * c * 2 if a[3] else 0  # the shortcut gradient summed in (MAXPOOL_LINK)
        return ("maxpool bwd" + (" + linked dy" if a[3] else ""), n * ho * wo * c * 3 + linked + n * h * w * c * 2, 0)

    for name, model in [("det_bn_fwd_train", bn_fwd_train), ("det_bn_stats_train", bn_stats),
                        ("det_bn_fwd_from_partials", bn_fwd_parts), ("det_bn_apply", bn_apply),
                        ("det_bn_apply_res_mbits", bn_apply_res_mbits), ("det_bn_bwd", bn_bwd),
                        ("det_bn_bwd_from_partials", bn_bwd_parts), ("det_bn_bwd_finalize_partials", bn_bwd_fin),
                        ("det_bn_bwd_apply_coef", bn_bwd_coef), ("det_conv_nt", conv_nt), ("det_conv_dgrad", conv_dgrad),
                        ("det_conv_nt_bnbwd", conv_nt_bnbwd), ("det_conv_tn", conv_tn), ("det_conv_wgrad", conv_wgrad),
                        ("det_igemm_wgrad", igemm_wgrad), ("det_igemm_conv_cfg", igemm_conv),
                        ("det_igemm_conv_bnbwd", igemm_bnbwd), ("det_igemm_dgrad_s2", dgrad_s2), ("det_conv3p", conv3p),
                        ("det_conv3p_wgrad", conv3p_wgrad), ("det_stem_conv_fwd", stem_fwd), ("det_stemp_wgrad", stemp),
                        ("det_conv_dgrad_weight", dgrad_weight), ("det_maxpool3s2_fwd", maxpool_fwd),
                        ("det_maxpool3s2_bwd", maxpool_bwd)]:
        wrap(name, model)

    from determined_1_amd.models import resnet
    from determined_1_amd.ops.functional import u8_normalize
    from determined_1_amd.models.synthetic import IMAGENET_MEAN, IMAGENET_STD

    torch.manual_seed(0)
    model = resnet.resnet50(num_classes=1000).to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16)
    for mod in model.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.float()
    img = torch.randint(0, 256, (args.batch, args.image_size, args.image_size, 3), dtype=torch.uint8, device=dev)
    y = torch.randint(0, 1000, (args.batch,), device=dev)

    def step():
        model.zero_grad(set_to_none=True)
        x = u8_normalize(img, IMAGENET_MEAN, IMAGENET_STD, out_dtype=torch.bfloat16, pad4=True)
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
    per = len(recs) // args.iters
    rows = []
    for i in range(per):
        grp = [recs[i + j * per] for j in range(args.iters)]
        name, kind, nb, fl = grp[0][:4]
        ms = sum(g[4].elapsed_time(g[5]) for g in grp) / len(grp)
        tbs = nb / (ms * 1e-3) / 1e12
        ref = copy_tbs(dev, nb)
        rows.append((i, name, kind, nb, fl, ms, tbs, 100 * tbs / ref, ref, fl / (ms * 1e-3) / 1e12 if fl else 0.0))
    fam = defaultdict(lambda: [0, 0.0, 0, 0.0, 0.0])
    for r in rows:
        f = fam[r[2]]
        f[0] += 1
        f[1] += r[5]
        f[2] += r[3]
        f[3] += r[4]
        f[4] += r[3] / (r[8] * 1e12) * 1e3  # ms a same-size copy would take
    print(f"{'#':>3} {'kernel family':<44} {'MB':>9} {'ms':>7} {'TB/s':>6} {'%copy':>6} {'TF/s':>7}")
    for r in rows:
        print(f"{r[0]:>3} {r[2]:<44} {r[3] / 1e6:>9.1f} {r[5]:>7.3f} {r[6]:>6.2f} {r[7]:>6.1f} {r[9]:>7.1f}")
    print("\nper family (sum over the step): calls, ms, GB, TB/s, % of same-size copies, TF/s")
    tot_ms = sum(f[1] for f in fam.values())
    for k, f in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:<46} {f[0]:>3} {f[1]:>7.3f} {f[2] / 1e9:>6.2f} {f[2] / (f[1] * 1e-3) / 1e12:>6.2f} "
              f"{100 * f[4] / f[1]:>6.1f} {f[3] / (f[1] * 1e-3) / 1e12:>7.1f}")
    print(f"  {'TOTAL native calls':<46} {len(rows):>3} {tot_ms:>7.3f}")
    if args.out:
        with open(args.out, "w", newline="") as fo:
            w = csv.writer(fo)
            w.writerow(["idx", "entry", "family", "bytes", "flops", "ms", "TB_s", "pct_of_same_size_copy",
                        "copy_TB_s", "TF_s"])
            for r in rows:
                w.writerow([r[0], r[1], r[2], r[3], r[4], f"{r[5]:.4f}", f"{r[6]:.3f}", f"{r[7]:.1f}", f"{r[8]:.2f}",
                            f"{r[9]:.1f}"])
            for k, f in sorted(fam.items(), key=lambda kv: -kv[1][1]):
                w.writerow(["family", "", k, f[2], f[3], f"{f[1]:.4f}", f"{f[2] / (f[1] * 1e-3) / 1e12:.3f}",
                            f"{100 * f[4] / f[1]:.1f}", "", f"{f[3] / (f[1] * 1e-3) / 1e12:.1f}"])


if __name__ == "__main__":
    main()
