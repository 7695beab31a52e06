#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit $?
timeout -k 10 400 python scripts/microbench_conv.py 0 > gpurun_out/mb_conv0.log 2>&1 || exit $?
timeout -k 10 500 python scripts/microbench_conv.py 1 > gpurun_out/mb_conv1.log 2>&1 || exit $?
DET_BENCH_CUDNN_BENCHMARK=1 timeout -k 10 400 python bench.py > gpurun_out/bench_cudnnbench.log 2>&1 || exit $?
DET_BENCH_BS=512 timeout -k 10 400 python bench.py > gpurun_out/bench_bs512.log 2>&1 || exit $?
echo done
