#!/bin/bash
# Round-2 session 9: re-verify the restored tree on a fresh box: full GPU test tier + 1-GPU bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s9
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/s9/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/s9/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/s9/pytest_gpu.log
timeout -k 10 400 python -u bench.py > gpurun_out/s9/bench.json 2> gpurun_out/s9/bench.err || { tail -20 gpurun_out/s9/bench.err; exit 1; }
cat gpurun_out/s9/bench.json
