#!/bin/bash
# Round-2 session 29: single-pass stem wgrad (K = 256 in one workgroup) numerics + bench; seed the
# MIOpen find-db / kernel cache for the bucketed DETR and Faster R-CNN shapes (harvested into
# gpurun_out/miopen_db for the repo), then the detection benches on the seeded db.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s29
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "stem or u8" > gpurun_out/s29/conv.log 2>&1 || { tail -40 gpurun_out/s29/conv.log; exit 1; }
tail -2 gpurun_out/s29/conv.log
timeout -k 10 400 python -u bench.py > gpurun_out/s29/bench.json 2> gpurun_out/s29/bench.err || { tail -20 gpurun_out/s29/bench.err; exit 1; }
cat gpurun_out/s29/bench.json
timeout -k 10 900 python -u scripts/miopen_seed_detection.py --harvest gpurun_out/miopen_db > gpurun_out/s29/seed.log 2>&1 || { tail -30 gpurun_out/s29/seed.log; exit 1; }
grep -v "^\[" gpurun_out/s29/seed.log | tail -6
for m in fasterrcnn detr; do
  for a in O2 O0; do
    timeout -k 10 300 python -u scripts/bench_detection.py --model $m --steps 30 --warmup 10 --amp $a > gpurun_out/s29/${m}_${a}.json 2> gpurun_out/s29/${m}_${a}.err || { tail -30 gpurun_out/s29/${m}_${a}.err; exit 1; }
    cat gpurun_out/s29/${m}_${a}.json
  done
done
