"""Measure vendor-BLAS solutions for a workload's GEMMs and merge them into the shipped file
(determined_1_amd/ops/tuned/gemm_gfx950.csv, loaded read-only by ops/gemm_tuning.py).

    python scripts/tune_gemms.py -- python scripts/bench_bert.py --steps 3 --warmup 2

Runs the command once (on an MI355X) with PyTorch TunableOp tuning on -- every hipBLASLt and rocBLAS
solution of each new GEMM shape is timed and the fastest kept -- then merges the results: a shape
already in the file keeps whichever entry is faster.  The validator lines (torch / HIP / hipBLASLt /
rocBLAS versions, GPU arch) must match the file's, since TunableOp ignores entries from another stack.
"""
import argparse
import glob
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIPPED = os.path.join(REPO, "determined_1_amd", "ops", "tuned", "gemm_gfx950.csv")


def read(path):
    val, ent = {}, {}
    with open(path) as f:
        for line in f:
            p = line.rstrip("\n").split(",")
            if len(p) < 3:
                continue
            if p[0] == "Validator":
                val[p[1]] = ",".join(p[2:])
            else:
                ent[(p[0], p[1])] = (p[2], float(p[3]) if len(p) > 3 else float("inf"))
    return val, ent


def merge(new_path, out_path=SHIPPED):
    nv, ne = read(new_path)
    if os.path.exists(out_path):
        ov, oe = read(out_path)
        if ov != nv:
            raise SystemExit(f"validators differ ({ov} vs {nv}): re-tune every shape on this stack instead")
    else:
        ov, oe = nv, {}
    for k, v in ne.items():
        if k not in oe or v[1] < oe[k][1]:
            oe[k] = v
    with open(out_path, "w") as f:
        for k, v in nv.items():
            f.write(f"Validator,{k},{v}\n")
        for (op, shape), (sol, t) in sorted(oe.items()):
            f.write(f"{op},{shape},{sol},{t}\n")
    return len(oe)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    ap.add_argument("--out", default=SHIPPED)
    args = ap.parse_args()
    cmd = args.cmd[1:] if args.cmd and args.cmd[0] == "--" else args.cmd
    if not cmd:
        raise SystemExit("usage: tune_gemms.py -- <command>")
    d = tempfile.mkdtemp(prefix="det-tune-")
    env = dict(os.environ, PYTORCH_TUNABLEOP_ENABLED="1", PYTORCH_TUNABLEOP_TUNING="1",
               PYTORCH_TUNABLEOP_FILENAME=os.path.join(d, "tuned.csv"), DET_TUNED_GEMMS="0")
    rc = subprocess.call(cmd, env=env)
    if rc != 0:
        raise SystemExit(rc)
    files = glob.glob(os.path.join(d, "tuned*.csv"))
    if not files:
        raise SystemExit("the command ran no tunable GEMM")
    for f in files:
        n = merge(f, args.out)
    print(f"{args.out}: {n} shapes")


if __name__ == "__main__":
    sys.exit(main())
