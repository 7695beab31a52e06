#!/bin/bash
# Round-2 session 30: round-end rehearsal on the final tree: full GPU test tier, smoke(), 1-GPU bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s30
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/s30/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s30/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/s30/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s30/smoke.log 2>&1 || { tail -20 gpurun_out/s30/smoke.log; exit 1; }
tail -1 gpurun_out/s30/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/s30/bench.json 2> gpurun_out/s30/bench.err || { tail -20 gpurun_out/s30/bench.err; exit 1; }
cat gpurun_out/s30/bench.json
timeout -k 10 300 python -u scripts/bench_stem.py > gpurun_out/s30/stem_occ2.jsonl 2> gpurun_out/s30/stem.err || { tail -20 gpurun_out/s30/stem.err; exit 1; }
cat gpurun_out/s30/stem_occ2.jsonl
DET_STEM_OCC=3 timeout -k 10 300 python -u scripts/bench_stem.py > gpurun_out/s30/stem_occ3.jsonl 2> gpurun_out/s30/stem3.err || { tail -20 gpurun_out/s30/stem3.err; exit 1; }
cat gpurun_out/s30/stem_occ3.jsonl
# detection on a fresh box from the shipped (in-tree) seeded MIOpen db
for m in fasterrcnn detr; do
  timeout -k 10 300 python -u scripts/bench_detection.py --model $m --steps 30 --warmup 10 --amp O0 > gpurun_out/s30/${m}_O0.json 2> gpurun_out/s30/${m}_O0.err || { tail -30 gpurun_out/s30/${m}_O0.err; exit 1; }
  cat gpurun_out/s30/${m}_O0.json
done
