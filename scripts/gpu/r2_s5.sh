#!/bin/bash
# Round-2 session 5: two-stage BN finalize + K=64 single-buffer GEMM variant: numerics, conv
# microbench, BN roofline table, ResNet-50 bench and steady-state kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s5
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_norm_gpu.py > gpurun_out/s5/pytest.log 2>&1; rc=$?
[ $rc -le 1 ] || { tail -30 gpurun_out/s5/pytest.log; exit 1; }
tail -3 gpurun_out/s5/pytest.log
timeout -k 10 300 python -u scripts/bench_conv1x1.py 512 > gpurun_out/s5/conv1x1.jsonl 2> gpurun_out/s5/conv1x1.err || { tail -20 gpurun_out/s5/conv1x1.err; exit 1; }
tail -1 gpurun_out/s5/conv1x1.jsonl
timeout -k 10 300 python -u scripts/bn_roofline.py --out gpurun_out/s5/bn_bandwidth.csv > gpurun_out/s5/bn_roofline.txt 2>&1 || { tail -20 gpurun_out/s5/bn_roofline.txt; exit 1; }
tail -3 gpurun_out/s5/bn_roofline.txt
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s5/bench.json 2> gpurun_out/s5/bench.err || { tail -20 gpurun_out/s5/bench.err; exit 1; }
cat gpurun_out/s5/bench.json
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d gpurun_out/s5/prof -o run -- python3 -u bench.py --steps 10 --warmup 5 > gpurun_out/s5/bench_prof.json 2> gpurun_out/s5/bench_prof.err || { tail -20 gpurun_out/s5/bench_prof.err; exit 1; }
