#!/bin/bash
# Round-6 session 79: final rehearsal (4) -- the whole GPU suite after the capture / RCCL event-cache hardening,
# smoke(), and bench.py with its defaults (1,024 images/GPU, eager + side stream) twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s79
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.log 2>&1
rc=$?; tail -2 $O/gpu_suite.log; grep -E "FAILED|ERROR" $O/gpu_suite.log | head -30
grep -q -E "Fatal Python|Segmentation fault" $O/gpu_suite.log && exit 3
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $O/bench$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo "bench: $(cut -c1-150 $O/bench$i.json)"
done
