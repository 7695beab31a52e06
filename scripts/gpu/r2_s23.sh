#!/bin/bash
# Round-2 session 23: round-end rehearsal on the current tree: full GPU tier, smoke(), 1-GPU bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s23
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/s23/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s23/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/s23/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s23/smoke.log 2>&1 || { tail -30 gpurun_out/s23/smoke.log; exit 1; }
tail -1 gpurun_out/s23/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/s23/bench.json 2> gpurun_out/s23/bench.err || { tail -20 gpurun_out/s23/bench.err; exit 1; }
cat gpurun_out/s23/bench.json
