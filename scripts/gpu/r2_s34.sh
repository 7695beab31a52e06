#!/bin/bash
# Round-2 session 34: RetinaNet R50-FPN (mmdetection retinanet.yaml stand-in): example on the GPU,
# find-db seeding for its bucket shapes (harvested), throughput fp32 / bf16.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s34
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_examples_gpu.py -k "retinanet or maskrcnn" > gpurun_out/s34/test.log 2>&1 || { tail -40 gpurun_out/s34/test.log; exit 1; }
tail -2 gpurun_out/s34/test.log
timeout -k 10 600 python -u scripts/miopen_seed_detection.py --models retinanet --harvest gpurun_out/miopen_db > gpurun_out/s34/seed.log 2>&1 || { tail -30 gpurun_out/s34/seed.log; exit 1; }
grep -v "^\[" gpurun_out/s34/seed.log | tail -4
for a in O0 O2; do
  timeout -k 10 300 python -u scripts/bench_detection.py --model retinanet --steps 30 --warmup 10 --amp $a > gpurun_out/s34/retinanet_${a}.json 2> gpurun_out/s34/retinanet_${a}.err || { tail -30 gpurun_out/s34/retinanet_${a}.err; exit 1; }
  cat gpurun_out/s34/retinanet_${a}.json
done
