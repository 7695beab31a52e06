#!/bin/bash
# Round-5 session 42: rebuilt container -- the whole GPU suite + smoke() on the fresh build, then
# bench.py (ResNet-50) twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s42
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.log 2>&1
rc=$?; tail -3 $O/gpu_suite.log; grep -E "FAILED|ERROR" $O/gpu_suite.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $O/bench$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo "bench: $(cut -c1-200 $O/bench$i.json)"
done
