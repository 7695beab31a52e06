"""GPU-busy fraction of a multi-process run from rocprofv3 kernel traces: the union of every kernel
interval in every process's database under DIR, over the window from the first to the last kernel
(the ASHA benchmark: one trial process per container, run under ``rocprofv3 --kernel-trace``).

    python scripts/prof_busy.py DIR [--out summary.json]
"""
import argparse
import glob
import json
import os
import sqlite3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    iv, per = [], []
    for db in sorted(glob.glob(os.path.join(args.dir, "**", "*.db"), recursive=True)):
        try:
            rows = sqlite3.connect(db).execute("select start, end from kernels").fetchall()
        except sqlite3.Error:
            continue
        if rows:
            iv.extend(rows)
            per.append({"db": os.path.relpath(db, args.dir), "kernels": len(rows),
                        "kernel_s": round(sum(e - s for s, e in rows) / 1e9, 3),
                        "span_s": round((max(e for _, e in rows) - min(s for s, _ in rows)) / 1e9, 3)})
    if not iv:
        raise SystemExit("no kernel rows found")
    iv.sort()
    busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    window = iv[-1][1] - iv[0][0] if iv else 0
    res = {"processes": len(per), "kernels": len(iv), "window_s": round(window / 1e9, 3),
           "gpu_busy_s": round(busy / 1e9, 3), "gpu_busy_frac": round(busy / max(window, 1), 4), "per_process": per}
    text = json.dumps(res, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")
    print(json.dumps({k: v for k, v in res.items() if k != "per_process"}))


if __name__ == "__main__":
    main()
