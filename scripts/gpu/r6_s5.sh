#!/bin/bash
# Round-6 session 5: native conv2d for the detection backbones (exactness tests, Faster R-CNN A/B),
# then which RCCL collectives capture into a hipGraph (world 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_conv2d_native_gpu.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "FAILED|ERROR|Error|Fatal|Segmentation" $O/tests.log | head -20
[ $rc -le 1 ] || exit $rc
grep -q -E "Fatal Python|Segmentation|core dumped" $O/tests.log && exit 3
for nat in 1 0; do
  DET_NATIVE_CONV2D=$nat timeout -k 10 400 python -u scripts/bench_detection.py --model fasterrcnn --amp O2 --steps 30 --warmup 10 > $O/frcnn_native$nat.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  echo "frcnn native=$nat: $(cut -c1-250 $O/frcnn_native$nat.json)"
done
NCCL_DEBUG=WARN timeout -k 10 400 python -u scripts/dbg/rccl_capture.py > $O/capture.jsonl 2> $O/capture.err
rc=$?; echo "capture rc=$rc"; cut -c1-400 $O/capture.jsonl
exit $rc
