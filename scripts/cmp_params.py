"""Compare two ``--params-out`` files (bench.py / scripts/bench_bert.py): max relative difference of
the per-tensor sums and norms.  python scripts/cmp_params.py A.pt B.pt [--tol 1e-3]"""
import json
import sys

import torch


def main() -> None:
    a, b = torch.load(sys.argv[1], weights_only=True), torch.load(sys.argv[2], weights_only=True)
    tol = float(sys.argv[sys.argv.index("--tol") + 1]) if "--tol" in sys.argv else 1e-3
    out = {}
    for k in ("sums", "norms"):
        d = (a[k] - b[k]).abs() / (b[k].abs() + 1e-12)
        out[k + "_max_rel"] = float(d.max())
        out[k + "_exact"] = bool(torch.equal(a[k], b[k]))
    out["graph_b"] = b.get("graph")
    out["ok"] = out["norms_max_rel"] <= tol
    print(json.dumps(out))
    sys.exit(0 if out["ok"] else 1)


if __name__ == "__main__":
    main()
