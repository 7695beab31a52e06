#!/bin/bash
# Session: linked projection-shortcut conv (dgrad summed in the producer's BN backward): numerics,
# then the 1-GPU bench and the bare-loop harness-overhead comparison.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_norm_gpu.py tests/test_smoke_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_s32.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_s32.log | tail -20
grep -B2 -A20 "Error" gpurun_out/pytest_s32.log | head -50
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 420 python -u bench.py > gpurun_out/bench_s32.log 2>&1 || { echo "bench failed $?"; tail -30 gpurun_out/bench_s32.log; exit 1; }
grep '^{' gpurun_out/bench_s32.log
timeout -k 10 300 python -u scripts/bench_bare.py > gpurun_out/bare_s32.log 2>&1 || { echo "bare failed $?"; tail -30 gpurun_out/bare_s32.log; exit 1; }
grep '^{' gpurun_out/bare_s32.log
