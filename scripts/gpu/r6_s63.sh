#!/bin/bash
# Round-6 session 63: eight-phase wgrad (cfg 14) as the default where it fits vs DET_WGRAD8=0, at
# 1,024 and 512 images/GPU (bench defaults otherwise), alternating; then the conv GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s63
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv3x3_gpu.py tests/test_wgrad_stream_gpu.py \
  > $O/test.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error" $O/test.log | head; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for rep in 1 2; do
  for bs in 1024 512; do
    for v in 0 1; do
      DET_WGRAD8=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --batch-per-gpu $bs > $O/b.json 2> $O/b.err \
        || { echo "bench wgrad8=$v bs=$bs rc=$?"; tail -20 $O/b.err; exit 1; }
      line=$(grep '^{' $O/b.json | tail -1)
      echo "{\"wgrad8\": $v, \"bs\": $bs, \"bench\": $line}" >> $O/ab.jsonl
      echo "bs=$bs wgrad8=$v: $(echo "$line" | grep -o '"value": [0-9.]*')"
    done
  done
done
