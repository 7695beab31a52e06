#!/bin/bash
# Session: full GPU test tier + smoke() + default 1-GPU bench on the current tree (round-end rehearsal).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_s34.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed" gpurun_out/pytest_s34.log | tail -3
grep -E "FAILED|Error" gpurun_out/pytest_s34.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_s34.log 2>&1 || { echo "smoke failed $?"; tail -20 gpurun_out/smoke_s34.log; exit 1; }
tail -1 gpurun_out/smoke_s34.log
timeout -k 10 420 python -u bench.py > gpurun_out/bench_s34.log 2>&1 || { echo "bench failed $?"; tail -30 gpurun_out/bench_s34.log; exit 1; }
grep '^{' gpurun_out/bench_s34.log
