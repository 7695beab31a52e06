#!/bin/bash
# Round-4 session 26 (end of round): the whole GPU test tier as the driver runs it, smoke(), the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s26
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 900 --timeout-method thread -o faulthandler_timeout=300 -p no:cacheprovider -m gpu > $O/pytest_gpu.log 2>&1 || { grep -E "PASSED|FAILED|ERROR" $O/pytest_gpu.log | tail -5; tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -30 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
