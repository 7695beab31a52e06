#!/bin/bash
# Round-2 session 26 (rebuilt container): bn2->conv3 GEMM-prologue fusion numerics, full GPU tier
# incl. the detection kernels and the DETR / Faster R-CNN examples, smoke(), 1-GPU ResNet-50 bench
# A/B (bn prologue on/off), detection training throughput (fp32 + bf16 O2).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s26
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_detect_gpu.py tests/test_conv_gpu.py "tests/test_examples_gpu.py" -k "detect or roi or nms or conv or bn_relu or detr or fasterrcnn" > gpurun_out/s26/conv.log 2>&1 || { tail -40 gpurun_out/s26/conv.log; exit 1; }
tail -2 gpurun_out/s26/conv.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/s26/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s26/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/s26/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s26/smoke.log 2>&1 || { tail -20 gpurun_out/s26/smoke.log; exit 1; }
tail -1 gpurun_out/s26/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/s26/bench.json 2> gpurun_out/s26/bench.err || { tail -20 gpurun_out/s26/bench.err; exit 1; }
cat gpurun_out/s26/bench.json
timeout -k 10 400 python -u bench.py --no-bn-prologue > gpurun_out/s26/bench_noprologue.json 2> gpurun_out/s26/bench_noprologue.err || { tail -20 gpurun_out/s26/bench_noprologue.err; exit 1; }
cat gpurun_out/s26/bench_noprologue.json
for m in detr fasterrcnn; do
  for a in O0 O2; do
    timeout -k 10 300 python -u scripts/bench_detection.py --model $m --steps 30 --warmup 10 --amp $a > gpurun_out/s26/${m}_${a}.json 2> gpurun_out/s26/${m}_${a}.err || { tail -30 gpurun_out/s26/${m}_${a}.err; exit 1; }
    cat gpurun_out/s26/${m}_${a}.json
  done
done
timeout -k 10 300 python -u scripts/bench_stem.py > gpurun_out/s26/stem.jsonl 2> gpurun_out/s26/stem.err || { tail -20 gpurun_out/s26/stem.err; exit 1; }
cat gpurun_out/s26/stem.jsonl
