#!/bin/bash
# Round-5 session 34: the whole GPU suite (what the driver runs at round end) + smoke().
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s34
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1080 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.log 2>&1
rc=$?; tail -5 $O/gpu_suite.log; grep -E "FAILED|ERROR" $O/gpu_suite.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 $O/smoke.log
