#!/bin/bash
# Session: the whole GPU test tier (incl. the new DARTS-PTB / GAEA examples and the step-timer phases).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1050 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
echo "rc=$?"
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_all.log | tail -100 | grep -v PASSED
grep -c PASSED gpurun_out/pytest_all.log
grep -B5 -A25 "Error" gpurun_out/pytest_all.log | head -80
