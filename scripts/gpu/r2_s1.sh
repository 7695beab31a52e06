#!/bin/bash
# Round-2 session 1: RCCL world-1 data path + sum_rows numerics, then MIOpen warmup cold vs seeded.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s1
export DET_MIOPEN_DIR=$PWD/gpurun_out/s1/miopen
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rccl_gpu.py \
  "tests/test_kernels_gpu.py::test_sum_rows_fp32_accumulation" > gpurun_out/s1/pytest.log 2>&1 || { tail -40 gpurun_out/s1/pytest.log; exit 1; }
tail -3 gpurun_out/s1/pytest.log
# cold MIOpen db (fresh dir): warmup_s measures find-mode tuning
timeout -k 10 540 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s1/bench_cold.json 2> gpurun_out/s1/bench_cold.err || { tail -20 gpurun_out/s1/bench_cold.err; exit 1; }
cat gpurun_out/s1/bench_cold.json
# same db, new process: find results come from the user db
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s1/bench_warm.json 2> gpurun_out/s1/bench_warm.err || { tail -20 gpurun_out/s1/bench_warm.err; exit 1; }
cat gpurun_out/s1/bench_warm.json
du -sh gpurun_out/s1/miopen/* ; ls -la gpurun_out/s1/miopen/db gpurun_out/s1/miopen/cache
