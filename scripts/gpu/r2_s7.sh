#!/bin/bash
# Round-2 session 7: det_igemm 4-wave (128x64 wave tiles) vs 8-wave variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s7
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_igemm_gpu.py > gpurun_out/s7/pytest_igemm.log 2>&1 || { tail -30 gpurun_out/s7/pytest_igemm.log; exit 1; }
tail -2 gpurun_out/s7/pytest_igemm.log
timeout -k 10 300 python -u scripts/bench_igemm.py 512 > gpurun_out/s7/igemm4.jsonl 2> gpurun_out/s7/igemm4.err || { tail -20 gpurun_out/s7/igemm4.err; exit 1; }
DET_IGEMM_WAVES=8 timeout -k 10 300 python -u scripts/bench_igemm.py 512 > gpurun_out/s7/igemm8.jsonl 2> gpurun_out/s7/igemm8.err || { tail -20 gpurun_out/s7/igemm8.err; exit 1; }
tail -1 gpurun_out/s7/igemm4.jsonl; tail -1 gpurun_out/s7/igemm8.jsonl
