#!/bin/bash
# Session: all examples' local test mode on the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_examples_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_ex.log 2>&1
echo "rc=$?"
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_ex.log | tail -12
grep -B5 -A25 "Error" gpurun_out/pytest_ex.log | head -60
