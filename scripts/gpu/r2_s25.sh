#!/bin/bash
# Detection kernels (RoIAlign / NMS) numerics, DETR + Faster R-CNN examples on the MI355X, training
# throughput at the reference configs, fp32 (reference precision) and bf16 O2.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_detect_gpu.py > gpurun_out/s25_detect.log 2>&1 || { tail -60 gpurun_out/s25_detect.log; exit 1; }
tail -3 gpurun_out/s25_detect.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -k "detr or fasterrcnn" tests/test_examples_gpu.py > gpurun_out/s25_test.log 2>&1 || { tail -40 gpurun_out/s25_test.log; exit 1; }
tail -3 gpurun_out/s25_test.log
for m in detr fasterrcnn; do
  for a in O0 O2; do
    timeout -k 10 300 python -u scripts/bench_detection.py --model $m --steps 30 --warmup 10 --amp $a > gpurun_out/s25_${m}_${a}.json 2> gpurun_out/s25_${m}_${a}.err || { tail -30 gpurun_out/s25_${m}_${a}.err; exit 1; }
    cat gpurun_out/s25_${m}_${a}.json
  done
done
