#!/bin/bash
# Session: ResNet-50 bs512 kernel trace (ordering of MIOpen fills / SubTensorOp vs conv kernels).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o r50 --output-format csv -- python3 bench.py --steps 4 --warmup 8 > gpurun_out/prof_r50.log 2>&1
echo "rc=$?"
grep metric gpurun_out/prof_r50.log | cut -c1-150
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_r50/r50_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# keep the last 4 steps: from the 4th-from-last occurrence of the optimizer kernel
opt = [i for i, r in enumerate(rows) if "opt_kernel" in r["Kernel_Name"] or "sgd" in r["Kernel_Name"].lower()]
start = opt[-5] + 1 if len(opt) >= 5 else 0
with open("gpurun_out/r50_last_step_seq.csv", "w") as f:
    w = csv.writer(f)
    w.writerow(["idx", "dur_us", "grid", "name"])
    for i, r in enumerate(rows[opt[-2] + 1: opt[-1] + 1] if len(opt) >= 2 else rows[-400:]):
        w.writerow([i, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r.get("Grid_Size", ""), r["Kernel_Name"][:160]])
print("opt kernels", len(opt), "rows", len(rows))
PY
rm -f gpurun_out/prof_r50/r50_kernel_trace.csv
