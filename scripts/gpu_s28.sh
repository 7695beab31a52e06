#!/bin/bash
# Session: direct-landing numerics + 2-rank GPU-sharing BERT DP with aggregation.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_transformer_gpu.py tests/test_smoke_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_s28.log 2>&1
echo "rc=$?"
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_s28.log | tail -8
grep -B2 -A12 "Error" gpurun_out/pytest_s28.log | head -40
