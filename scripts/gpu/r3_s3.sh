#!/bin/bash
# Round-3 session 3: steady-state kernel tables, native 3x3 vs MIOpen 3x3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3s3
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3s3/prof_native -o run -- python3 -u bench.py --steps 10 --warmup 8 > gpurun_out/r3s3/bench_prof_native.json 2> gpurun_out/r3s3/bench_prof_native.err || { tail -20 gpurun_out/r3s3/bench_prof_native.err; exit 1; }
f=$(find gpurun_out/r3s3/prof_native -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out gpurun_out/r3s3/native_steady.csv > gpurun_out/r3s3/native_steady.txt 2>&1 || { tail -5 gpurun_out/r3s3/native_steady.txt; exit 1; }
head -45 gpurun_out/r3s3/native_steady.txt
rm -rf gpurun_out/r3s3/prof_native
