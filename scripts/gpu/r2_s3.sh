#!/bin/bash
# Round-2 session 3: det_conv GEMM numerics + per-shape microbench vs MIOpen; MIOpen find without
# the naive reference solvers (default find mode, and FAST find mode) on the seeded db.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s3
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > gpurun_out/s3/pytest_conv.log 2>&1; rc=$?
tail -25 gpurun_out/s3/pytest_conv.log
if [ $rc -eq 0 ]; then
  timeout -k 10 300 python -u scripts/bench_conv1x1.py 512 > gpurun_out/s3/conv1x1.jsonl 2> gpurun_out/s3/conv1x1.err || { tail -20 gpurun_out/s3/conv1x1.err; exit 1; }
  cat gpurun_out/s3/conv1x1.jsonl
fi
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s3/bench_nonaive.json 2> gpurun_out/s3/bench_nonaive.err || { tail -20 gpurun_out/s3/bench_nonaive.err; exit 1; }
cat gpurun_out/s3/bench_nonaive.json
MIOPEN_FIND_MODE=2 timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s3/bench_fast.json 2> gpurun_out/s3/bench_fast.err || { tail -20 gpurun_out/s3/bench_fast.err; exit 1; }
cat gpurun_out/s3/bench_fast.json
