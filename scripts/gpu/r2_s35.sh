#!/bin/bash
# Round-2 session 35: frozen-BN fold cached per conv (detection backbones): GPU example tests and
# DETR / Faster R-CNN throughput.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s35
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_examples_gpu.py tests/test_detect_gpu.py -k "detr or rcnn or retinanet or roi or nms" > gpurun_out/s35/test.log 2>&1 || { tail -40 gpurun_out/s35/test.log; exit 1; }
tail -2 gpurun_out/s35/test.log
for m in detr fasterrcnn; do
  for a in O0 O2; do
    timeout -k 10 300 python -u scripts/bench_detection.py --model $m --steps 30 --warmup 10 --amp $a > gpurun_out/s35/${m}_${a}.json 2> gpurun_out/s35/${m}_${a}.err || { tail -30 gpurun_out/s35/${m}_${a}.err; exit 1; }
    cat gpurun_out/s35/${m}_${a}.json
  done
done
