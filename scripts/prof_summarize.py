"""Steady-state per-step kernel summary from a rocprofv3 kernel trace (CSV or rocpd ``.db``).

    python scripts/prof_summarize.py gpurun_out/prof/bench_kernel_trace.csv --step-kernel opt_kernel \
        [--skip-steps 3] [--out profiles/x.csv]

A "step" is delimited by the optimizer kernel (one fused launch per step).  Kernels before the end
of warmup (MIOpen find, first-iteration allocation) are dropped: the window starts after the
``--skip-steps``-th step kernel that follows the last ``naive_conv`` (find) dispatch.  Prints and
writes per-kernel ms/step, calls/step, share, and the GPU busy time vs wall time of the window.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    m = re.search(r"(bn_\w+)(<[^(]*>)?", name)
    if m:
        return m.group(0)
    name = re.sub(r"\(.*", "", name).replace("void ", "")
    return name[:110]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step-kernel", default="opt_kernel")
    ap.add_argument("--skip-steps", type=int, default=3)
    ap.add_argument("--out")
    ap.add_argument("--sequence", action="store_true",
                    help="also print one mid-window step's kernel sequence (per-dispatch durations)")
    args = ap.parse_args()
    rows = []
    if args.trace.endswith(".db"):  # rocprofv3 >= 7 default output (rocpd sqlite)
        import sqlite3

        con = sqlite3.connect(args.trace)
        rows = [(int(s), int(e), n) for s, e, n in con.execute("select start, end, name from kernels")]
    else:
        with open(args.trace) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    last_find = max((i for i, r in enumerate(rows) if "naive_conv" in r[2]), default=-1)
    # one step = the run of consecutive optimizer launches (one per arena) that ends it
    steps = [i for i, r in enumerate(rows) if args.step_kernel in r[2] and i > last_find
             and not (i + 1 < len(rows) and args.step_kernel in rows[i + 1][2])]
    if len(steps) <= args.skip_steps + 1:
        raise SystemExit(f"only {len(steps)} step kernels after warmup")
    lo, hi = steps[args.skip_steps], steps[-1]
    n_steps = len(steps) - 1 - args.skip_steps
    win = rows[lo + 1:hi + 1]
    agg = defaultdict(lambda: [0, 0])
    busy = 0
    for s, e, n in win:
        agg[short(n)][0] += e - s
        agg[short(n)][1] += 1
        busy += e - s
    wall = rows[hi][1] - rows[lo][1]
    # time with at least one kernel running: with kernels on two streams (side-stream weight
    # gradients) the per-kernel sum exceeds the wall and each overlapped kernel runs slower
    occupied, cur_s, cur_e = 0, None, None
    for s, e, _ in sorted(win):
        if cur_e is None or s > cur_e:
            occupied += 0 if cur_e is None else cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    occupied += 0 if cur_e is None else cur_e - cur_s
    out = sorted(agg.items(), key=lambda kv: -kv[1][0])
    print(f"steady-state window: {n_steps} steps, wall {wall / 1e6 / n_steps:.3f} ms/step, "
          f"kernel busy {busy / 1e6 / n_steps:.3f} ms/step ({100.0 * busy / max(1, wall):.1f}%), "
          f"occupied {occupied / 1e6 / n_steps:.3f} ms/step ({100.0 * occupied / max(1, wall):.1f}%)")
    for k, (t, c) in out[:40]:
        print(f"{t / 1e6 / n_steps:8.3f} ms/step {c / n_steps:6.1f}/step {100.0 * t / busy:5.1f}%  {k}")
    if args.sequence:
        mid = steps[args.skip_steps + n_steps // 2]
        nxt = steps[args.skip_steps + n_steps // 2 + 1]
        seq = rows[mid + 1:nxt + 1]
        print(f"one step ({len(seq)} kernels, {(rows[nxt][1] - rows[mid][1]) / 1e3:.1f} us):")
        for s0, e0, n0 in seq:
            print(f"  {(e0 - s0) / 1e3:8.2f} us  {short(n0)}")
    if args.out:
        with open(args.out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "ms_per_step", "calls_per_step", "percent_of_busy"])
            w.writerow(["__window__", f"{wall / 1e6 / n_steps:.4f}", n_steps, f"{100.0 * busy / max(1, wall):.2f}"])
            for k, (t, c) in out:
                w.writerow([k, f"{t / 1e6 / n_steps:.4f}", f"{c / n_steps:.2f}", f"{100.0 * t / busy:.2f}"])


if __name__ == "__main__":
    main()
