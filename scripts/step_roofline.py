"""Per-call roofline of every native kernel in a ResNet-50 training step ("a byte model
whose rows are all <= 100 % of measured copy bandwidth").

    python scripts/step_roofline.py [--batch 512] [--iters 3] [--out profiles/r4_step_roofline.csv]

Wraps the det_* entry points of libdetkernels.so with HIP events, runs forward + backward of the
benchmark's ResNet-50 (bf16 channels_last, fused BN, native convs), and for every call records its
compulsory bytes read and written (each tensor argument once -- re-reads that a kernel serves from
L2 / the 256 MiB Infinity Cache are not counted) and its FLOPs.  The bandwidth bound of each row is
the time the same reads and writes take as a pure read stream plus a pure write stream of those
sizes, measured on the same box (a reduction over, and a fill of, a freshly written buffer), so a
cache-resident small tensor is held to a cache-speed stream and a read-heavy kernel to the read
rate: rows above 100 % then mean the byte model is wrong.  Prints one row per call and a summary per kernel family."""
import argparse
import csv
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from determined_1_amd.ops import _lib  # noqa: E402

_BW = {}


def _bucket(nbytes: int) -> int:
    return max(1 << 20, 1 << int(nbytes).bit_length())  # power-of-two buckets


def stream_tbs(dev, nbytes: int, kind: str, lib=None) -> float:
    """Device bandwidth of a pure read ("r") or a pure write ("w") of ``nbytes`` (its power-of-two
    bucket) over a freshly written buffer (as a producer kernel leaves its output), on the tuned
    det_stream kernels (ops/csrc/det_stream.hip: 16 B/lane, several accesses in flight per lane;
    best of a few unroll x grid configurations and of plain / nontemporal accesses).  Round 4 used a
    BatchNorm statistics pass as the read stream, which read at only 3.6-4.9 TB/s and put rows
    above 100 %."""
    key = (kind, _bucket(nbytes))
    if key not in _BW:
        n = key[1]
        a = torch.empty(n // 4, dtype=torch.int32, device=dev)
        sink = torch.zeros(4, dtype=torch.int32, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st = torch.cuda.current_stream().cuda_stream
        best = 0.0
        for code in ((0, 5) if kind == "r" else (1, 2)):
            for unroll in (4, 8):
                for blocks in (4096, 8192):
                    ts = []
                    for _ in range(4):
                        a.fill_(1)
                        e0.record()
                        _lib.check(lib.det_stream(st, code, a.data_ptr(), a.data_ptr(), n, blocks, unroll, 3,
                                                  sink.data_ptr()), "det_stream")
                        e1.record()
                        torch.cuda.synchronize()
                        ts.append(e0.elapsed_time(e1))
                    ts.sort()
                    best = max(best, n / (ts[len(ts) // 2] * 1e-3) / 1e12)
        _BW[key] = best
    return _BW[key]


def ref_ms(dev, rb: int, wb: int, lib) -> float:
    """Time the same bytes take as a pure read plus a pure write of the same sizes."""
    ms = 0.0
    if rb:
        ms += rb / (stream_tbs(dev, rb, "r", lib) * 1e12) * 1e3
    if wb:
        ms += wb / (stream_tbs(dev, wb, "w", lib) * 1e12) * 1e3
    return ms


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.get_lib()
    raw = lib  # (the same object; the reference runs while the wrappers are switched off)
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
            kind, rb, wb, flops = model(a)
            recs.append((name, kind, (rb, wb), flops, e0, e1))
            return rc

        setattr(lib, name, call)

    el = lambda dt: 2 if dt == 1 else 4  # noqa: E731

    # Each model returns (family, bytes read, bytes written, flops): every tensor argument read or
    # written once.
    # ---- BatchNorm family (det_norm.hip)
    def bn_fwd_train(a):
        m, c, n = a[5], a[6], a[5] * a[6] * el(a[1])
        return ("bn fwd (stats+apply)", 2 * n + (n if a[3] else 0), n + (m * c // 8 if a[20] else 0), 0)

    def bn_stats(a):
        return ("bn stats", a[3] * a[4] * el(a[1]), 0, 0)

    def bn_fwd_parts(a):
        m, c, nrb, n = a[5], a[6], a[8], a[5] * a[6] * el(a[1])
        if not a[19]:
            return ("bn fwd finalize", 2 * nrb * c * 4, 0, 0)
        kind = "bn fwd finalize + apply" + (" (shortcut BN in the residual)" if a[26] else "")
        return (kind, 2 * nrb * c * 4 + n + (n if a[3] else 0), n + (m * c // 8 if a[24] else 0), 0)

    def bn_apply(a):
        n = a[5] * a[6] * el(a[1])
        return ("bn apply (frozen / deferred shortcut BN)", n + (n if a[3] else 0), n, 0)

    def bn_apply_res_mbits(a):
        m, c = a[4], a[5]
        return ("bn apply + res + mask (deferred)", 2 * m * c * 2, m * c * 2 + m * c // 8, 0)

    def bn_bwd(a):
        m, c, mode, n = a[6], a[7], a[8], a[6] * a[7] * el(a[1])
        # partial pass (dy [+dy2], x [+mbits]) then apply pass (the same again, writes dx [+dres])
        rd = n + (n if a[3] else 0) + n + (m * c // 8 if mode == 2 and a[5] else 0)
        if len(a) > 19 and not a[19]:  # apply deferred into the consuming GEMM: the partial pass only
            return (f"bn bwd partials (apply deferred) mask{mode}", rd, 0, 0)
        return (f"bn bwd (partials+apply) mask{mode}", 2 * rd, n + (n if a[15] else 0), 0)

    def bn_bwd_parts(a):
        m, c, nrb, n = a[4], a[5], a[11], a[4] * a[5] * el(a[1])
        return ("bn bwd finalize + apply", 2 * n + 2 * nrb * c * 4, n, 0)

    def bn_bwd_fin(a):
        return ("bn bwd finalize", 2 * a[8] * a[2] * 4, 0, 0)  # (nrb, rpb) = a[8], a[9]

    def bn_bwd_coef(a):
        n = a[4] * a[5] * el(a[1])
        return ("bn bwd apply (materialised)", 2 * n, n, 0)

    # ---- convolutions (det_conv.hip / det_igemm.hip)
    def conv_nt(a):
        m, n, k = a[4], a[5], a[6]
        gather = a[11] > 0
        rd, wr = m * k * 2 + n * k * 2, m * n * 2
        kind = "1x1 fwd" + (" s2" if gather else "") + (" +stats" if a[9] else "") + (" +prologue" if a[7] else "")
        if a[15]:  # AFWD: also reads the residual, writes the applied A and its mask bits (first N tile)
            rd += m * k * 2
            wr += m * k * 2 + m * k // 8
            kind = "1x1 fwd + bn3 apply (AFWD)"
        return (kind, rd, wr, 2 * m * n * k)

    def conv_dgrad(a):
        m, n, k = a[4], a[5], a[6]
        rd, wr = m * k * 2 + n * k * 2, m * n * 2
        if a[7]:
            rd += m * k * 2
            wr += m * k * 2
        return ("1x1 dgrad" + (" + bn bwd apply (ABN)" if a[7] else ""), rd, wr, 2 * m * n * k)

    def conv_nt_bnbwd(a):
        m, n, k, mode = a[4], a[5], a[6], a[15]
        rd, wr = m * k * 2 + n * k * 2 + m * n * 2, m * n * 2  # dY, W, bn x; write d
        if a[12]:
            rd += m * n * 2 // 4 if a[22] > 0 else m * n * 2  # shortcut gradient (stride-2 grid: a quarter)
        if mode == 2:
            rd += m * n // 8
        if a[17]:
            rd += m * k * 2
            wr += m * k * 2
        return (f"1x1 dgrad + bn bwd epilogue mask{mode}" + (" + ABN" if a[17] else ""), rd, wr, 2 * m * n * k)

    def conv_tn(a):
        m, n, k = a[5], a[6], a[7]
        return ("1x1 wgrad (gemm_tn)", m * n * 2 + m * k * 2, n * k * 4, 2 * m * n * k)

    def conv_wgrad(a):
        m, n, cin, r, s = a[5], a[6], a[7], a[12], a[13]
        hi, wi, ho, wo = a[8], a[9], a[10], a[11]
        x = (m // (ho * wo)) * hi * wi * cin * 2
        return (f"{r}x{s} wgrad (gemm_tn im2col)", m * n * 2 + x, n * r * s * cin * 4, 2 * m * n * r * s * cin)

    def igemm_wgrad(a):
        m, n, cin, r, s = a[5], a[6], a[7], a[12], a[13]
        hi, wi, ho, wo = a[8], a[9], a[10], a[11]
        x = (m // (ho * wo)) * hi * wi * cin * 2
        return (f"{r}x{s} wgrad (ring)", m * n * 2 + x, n * r * s * cin * 4, 2 * m * n * r * s * cin)

    def igemm_conv(a):
        m, n, cin, hi, wi, ho, wo, r, s = a[5], a[6], a[7], a[8], a[9], a[10], a[11], a[12], a[13]
        x = (m // (ho * wo)) * hi * wi * cin * 2
        kind = f"{r}x{s} s{a[14]} igemm" + (" +stats" if a[16] else "")
        return (kind, x + n * r * s * cin * 2, m * n * 2, 2 * m * n * r * s * cin)

    def igemm_bnbwd(a):
        m, n, cin, hi, wi, ho, wo, r, s = a[5], a[6], a[7], a[8], a[9], a[10], a[11], a[12], a[13]
        x = (m // (ho * wo)) * hi * wi * cin * 2
        return (f"{r}x{s} dgrad igemm + bn bwd epilogue", x + n * r * s * cin * 2 + m * n * 2, m * n * 2,
                2 * m * n * r * s * cin)

    def dgrad_s2(a):
        nb, ho, wo, cout, cin = a[5], a[6], a[7], a[8], a[9]
        m_in = nb * 4 * ho * wo
        rd = nb * ho * wo * cout * 2 + 9 * cin * cout * 2 + (m_in * cin * 2 if a[10] else 0)
        return ("3x3 s2 dgrad (parity classes)" + (" + bn bwd epilogue" if a[10] else ""), rd, m_in * cin * 2,
                2 * m_in * cin * cout * 9 // 4)

    def conv3p(a):
        nb, h, w, cin, n = a[4], a[5], a[6], a[7], a[8]
        m = nb * h * w
        kind = "3x3 conv3p" + (" dgrad + bn bwd epilogue" if a[13] else (" +stats" if a[11] else ""))
        return (kind, m * cin * 2 + 9 * n * cin * 2 + (m * n * 2 if a[13] else 0), m * n * 2, 2 * m * n * 9 * cin)

    def conv3p_wgrad(a):
        nb, h, w, cin, n = a[5], a[6], a[7], a[8], a[9]
        m = nb * h * w
        return ("3x3 wgrad (conv3p patch)", m * n * 2 + m * cin * 2, 9 * n * cin * 4, 2 * m * n * 9 * cin)

    def stem_fwd(a):
        m, hi, wi = a[4], a[5], a[6]
        nimg = m // (a[7] * a[8])
        return ("stem 7x7 fwd +stats", nimg * hi * wi * 8, m * 64 * 2, 2 * m * 64 * 147)

    def stemp(a):
        m, hi, wi, ho, wo = a[5], a[6], a[7], a[8], a[9]
        abn = len(a) > 12 and a[12]
        rd = m * 128 + (m // (ho * wo)) * hi * wi * 8 + (m * 128 if abn else 0)
        return ("stem wgrad (patch)" + (" + bn bwd apply (ABN)" if abn else ""), rd, 64 * 256 * 4, 2 * m * 64 * 147)

    def dgrad_weight(a):
        k, c, r, s = a[4], a[5], a[6], a[7]
        return ("dgrad weight flip", k * c * r * s * (2 if a[2] == 1 else 4), k * c * r * s * 2, 0)

    def maxpool_fwd(a):
        n, h, w, c = a[5], a[6], a[7], a[8]
        ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        return ("maxpool fwd", n * h * w * c * 2, n * ho * wo * c * 3, 0)

    def maxpool_bwd(a):
        n, h, w, c = a[6], a[7], a[8], a[9]
        ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        rd = n * ho * wo * c * 3 + (n * ho * wo * c * 2 if a[3] else 0)  # dy + idx (+ the linked dy2)
        bnb = len(a) > 10 and a[10]
        if bnb:
            rd += n * h * w * c * 2  # the BN input for the mask and the partial sums
        kind = "maxpool bwd" + (" + linked dy" if a[3] else "") + (" + bn bwd partials" if bnb else "")
        return (kind, rd, n * h * w * c * 2, 0)

    for name, model in [("det_bn_fwd_train", bn_fwd_train), ("det_bn_stats_train", bn_stats),
                        ("det_bn_fwd_from_partials", bn_fwd_parts), ("det_bn_apply", bn_apply),
                        ("det_bn_apply_res_mbits", bn_apply_res_mbits), ("det_bn_bwd", bn_bwd),
                        ("det_bn_bwd_from_partials", bn_bwd_parts), ("det_bn_bwd_finalize_partials", bn_bwd_fin),
                        ("det_bn_bwd_apply_coef", bn_bwd_coef), ("det_conv_nt", conv_nt), ("det_conv_dgrad", conv_dgrad),
                        ("det_conv_nt_bnbwd", conv_nt_bnbwd), ("det_conv_tn", conv_tn), ("det_conv_wgrad", conv_wgrad),
                        ("det_igemm_wgrad", igemm_wgrad), ("det_igemm_conv_cfg", igemm_conv),
                        ("det_igemm_conv_bnbwd", igemm_bnbwd), ("det_igemm_dgrad_s2", dgrad_s2), ("det_conv3p", conv3p),
                        ("det_conv3p_wgrad", conv3p_wgrad), ("det_stem_conv_fwd", stem_fwd), ("det_stemp_fwd", stem_fwd), ("det_stemp_wgrad", stemp),
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
        name, kind, (rb, wb), fl = grp[0][:4]
        ms = sum(g[4].elapsed_time(g[5]) for g in grp) / len(grp)
        nb = rb + wb
        tbs = nb / (ms * 1e-3) / 1e12
        rms = ref_ms(dev, rb, wb, raw)
        rows.append((i, name, kind, nb, fl, ms, tbs, 100 * rms / ms, rms, fl / (ms * 1e-3) / 1e12 if fl else 0.0, rb, wb))
    fam = defaultdict(lambda: [0, 0.0, 0, 0.0, 0.0])
    for r in rows:
        f = fam[r[2]]
        f[0] += 1
        f[1] += r[5]
        f[2] += r[3]
        f[3] += r[4]
        f[4] += r[8]  # ms the same reads + writes take as pure streams
    print(f"{'#':>3} {'kernel family':<48} {'MB rd':>8} {'MB wr':>8} {'ms':>7} {'TB/s':>6} {'%bw':>6} {'TF/s':>7}")
    for r in rows:
        print(f"{r[0]:>3} {r[2]:<48} {r[10] / 1e6:>8.1f} {r[11] / 1e6:>8.1f} {r[5]:>7.3f} {r[6]:>6.2f} {r[7]:>6.1f} "
              f"{r[9]:>7.1f}")
    print("\nper family (sum over the step): calls, ms, GB, TB/s, % of the streaming bound (the same reads and "
          "writes as pure read / write streams of those sizes), TF/s")
    tot_ms = sum(f[1] for f in fam.values())
    for k, f in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:<50} {f[0]:>3} {f[1]:>7.3f} {f[2] / 1e9:>6.2f} {f[2] / (f[1] * 1e-3) / 1e12:>6.2f} "
              f"{100 * f[4] / f[1]:>6.1f} {f[3] / (f[1] * 1e-3) / 1e12:>7.1f}")
    print(f"  {'TOTAL native calls':<50} {len(rows):>3} {tot_ms:>7.3f}")
    print("stream references (TB/s): " + ", ".join(f"{k[0]}{k[1] >> 20}MiB={v:.2f}" for k, v in sorted(_BW.items())))
    if args.out:
        with open(args.out, "w", newline="") as fo:
            w = csv.writer(fo)
            w.writerow(["idx", "entry", "family", "bytes_read", "bytes_written", "flops", "ms", "TB_s",
                        "pct_of_stream_bound", "stream_bound_ms", "TF_s"])
            for r in rows:
                w.writerow([r[0], r[1], r[2], r[10], r[11], r[4], f"{r[5]:.4f}", f"{r[6]:.3f}", f"{r[7]:.1f}",
                            f"{r[8]:.4f}", f"{r[9]:.1f}"])
            for k, f in sorted(fam.items(), key=lambda kv: -kv[1][1]):
                w.writerow(["family", "", k, f[2], "", f[3], f"{f[1]:.4f}", f"{f[2] / (f[1] * 1e-3) / 1e12:.3f}",
                            f"{100 * f[4] / f[1]:.1f}", f"{f[4]:.4f}", f"{f[3] / (f[1] * 1e-3) / 1e12:.1f}"])


if __name__ == "__main__":
    main()
