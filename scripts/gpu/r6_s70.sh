#!/bin/bash
# Round-6 session 70: detection trials (native backbone convs, bf16) with the side-stream weight
# gradients on (default) vs off (DET_WGRAD_STREAM=0), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s70
mkdir -p $O
export TMPDIR=/tmp
for m in fasterrcnn retinanet maskrcnn; do
  for v in 0 1 0 1; do
    DET_WGRAD_STREAM=$v timeout -k 10 400 python -u scripts/bench_detection.py --model $m --amp O2 --steps 30 --warmup 10 \
      > $O/d.json 2> $O/d.err || { echo "$m side=$v failed rc=$?"; tail -8 $O/d.err; exit 1; }
    line=$(grep '^{' $O/d.json | tail -1)
    echo "{\"model\": \"$m\", \"side\": $v, \"bench\": $line}" >> $O/det.jsonl
    echo "$m side=$v: $(echo "$line" | grep -o '"value": [0-9.]*')"
  done
done
