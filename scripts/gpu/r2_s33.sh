#!/bin/bash
# Round-2 session 33 (re-run after the RetinaNet commits as well): final rehearsal on the final tree (fresh box): full GPU test tier (incl. the
# Mask R-CNN example), smoke(), 1-GPU ResNet-50 bench, Mask R-CNN from the shipped find-db.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s33
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/s33/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s33/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/s33/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s33/smoke.log 2>&1 || { tail -20 gpurun_out/s33/smoke.log; exit 1; }
tail -1 gpurun_out/s33/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/s33/bench.json 2> gpurun_out/s33/bench.err || { tail -20 gpurun_out/s33/bench.err; exit 1; }
cat gpurun_out/s33/bench.json
timeout -k 10 300 python -u scripts/bench_detection.py --model maskrcnn --steps 30 --warmup 10 --amp O0 > gpurun_out/s33/maskrcnn_O0.json 2> gpurun_out/s33/maskrcnn_O0.err || { tail -30 gpurun_out/s33/maskrcnn_O0.err; exit 1; }
cat gpurun_out/s33/maskrcnn_O0.json
