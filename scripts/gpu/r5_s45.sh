#!/bin/bash
# Round-5 session 45: gap_bwd on 32-bit index math -- pool/conv GPU tests, smoke() and bench.py x2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s45
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pool_gpu.py tests/test_conv_gpu.py tests/test_conv3x3_gpu.py tests/test_dp_resnet_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $O/bench$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo "bench: $(cut -c1-150 $O/bench$i.json)"; cat $O/bench$i.json >> $O/bench.jsonl
done
