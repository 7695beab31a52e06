#!/bin/bash
# Round-2 session 27: native ResNet stem (det_conv implicit GEMM, 4-channel padded input, BN stats in
# the epilogue) numerics + ResNet-50 bench A/B + steady-state kernel profile; detection benches with
# shape bucketing (DETR pad_multiple 128, Faster R-CNN size_divisible 128).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s27
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py > gpurun_out/s27/conv.log 2>&1 || { tail -40 gpurun_out/s27/conv.log; exit 1; }
tail -2 gpurun_out/s27/conv.log
timeout -k 10 400 python -u bench.py > gpurun_out/s27/bench.json 2> gpurun_out/s27/bench.err || { tail -20 gpurun_out/s27/bench.err; exit 1; }
cat gpurun_out/s27/bench.json
timeout -k 10 400 python -u bench.py --no-native-stem > gpurun_out/s27/bench_nostem.json 2> gpurun_out/s27/bench_nostem.err || { tail -20 gpurun_out/s27/bench_nostem.err; exit 1; }
cat gpurun_out/s27/bench_nostem.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s27/prof -o run -- python -u bench.py --steps 10 --warmup 5 > gpurun_out/s27/prof_bench.json 2> gpurun_out/s27/prof_bench.err || { tail -20 gpurun_out/s27/prof_bench.err; exit 1; }
for m in detr fasterrcnn; do
  for a in O0 O2; do
    timeout -k 10 300 python -u scripts/bench_detection.py --model $m --steps 30 --warmup 10 --amp $a > gpurun_out/s27/${m}_${a}.json 2> gpurun_out/s27/${m}_${a}.err || { tail -30 gpurun_out/s27/${m}_${a}.err; exit 1; }
    cat gpurun_out/s27/${m}_${a}.json
  done
done
