#!/bin/bash
# Round-2 session 28: why is the Faster R-CNN trial step 3 s?  (a) one fixed image shape,
# (b) MIOpen FAST find mode with varying shapes, (c) kernel census of the fixed-shape run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s28
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/bench_detection.py --model fasterrcnn --steps 20 --warmup 5 --amp O2 --min-size 400 --max-size 400 > gpurun_out/s28/fixed.json 2> gpurun_out/s28/fixed.err || { tail -30 gpurun_out/s28/fixed.err; exit 1; }
cat gpurun_out/s28/fixed.json
MIOPEN_FIND_MODE=FAST timeout -k 10 300 python -u scripts/bench_detection.py --model fasterrcnn --steps 20 --warmup 5 --amp O2 > gpurun_out/s28/fast.json 2> gpurun_out/s28/fast.err || { tail -30 gpurun_out/s28/fast.err; exit 1; }
cat gpurun_out/s28/fast.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s28/prof -o run -- python -u scripts/bench_detection.py --model fasterrcnn --steps 10 --warmup 3 --amp O2 --min-size 400 --max-size 400 > gpurun_out/s28/prof.json 2> gpurun_out/s28/prof.err || { tail -30 gpurun_out/s28/prof.err; exit 1; }
cat gpurun_out/s28/prof.json
