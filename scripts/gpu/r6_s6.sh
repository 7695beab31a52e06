#!/bin/bash
# Round-6 session 6: native conv2d exactness (stride-2 1x1 with fp32 weights fixed), the RCCL capture
# probe over every collective, then the DP / aggregation hipGraph tests and the graph GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s6
mkdir -p $O
export TMPDIR=/tmp
NCCL_DEBUG=WARN timeout -k 10 400 python -u scripts/dbg/rccl_capture.py > $O/capture.jsonl 2> $O/capture.err
rc=$?; echo "capture rc=$rc"; cut -c1-300 $O/capture.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_conv2d_native_gpu.py tests/test_graph_dp_gpu.py tests/test_rccl_gpu.py tests/test_graph_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "FAILED|ERROR|Fatal|Segmentation|returncode=-" $O/tests.log | head -20
exit $rc
