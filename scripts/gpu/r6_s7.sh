#!/bin/bash
# Round-6 session 7: DP hipGraph capture on the capturing stream (thread_local capture mode), the BN
# one-launch finalizes (norm/BN tests, bench A/B), then the RCCL capture probe (crashing cases last).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_norm_gpu.py tests/test_bn_bwd_fusion_gpu.py tests/test_graph_dp_gpu.py tests/test_conv2d_native_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "FAILED|ERROR|Fatal|Segmentation|returncode=-" $O/tests.log | cut -c1-300 | head -20
[ $rc -le 1 ] || exit $rc
grep -q -E "returncode=-|Fatal Python|Segmentation fault" $O/tests.log && exit 3
for i in 1 2; do
  for lb in 1 0; do
    DET_BN_LASTBLOCK=$lb timeout -k 10 300 python -u bench.py > $O/bench_lb$lb.$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
    echo "bench lastblock=$lb: $(cut -c1-120 $O/bench_lb$lb.$i.json)"
  done
done
NCCL_DEBUG=WARN timeout -k 10 400 python -u scripts/dbg/rccl_capture.py > $O/capture.jsonl 2> $O/capture.err
echo "capture rc=$?"; cut -c1-300 $O/capture.jsonl
