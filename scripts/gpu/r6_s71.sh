#!/bin/bash
# Round-6 session 71: side-stream fork threshold (DET_WGRAD_STREAM_MIN, output-gradient elements) on
# the detection trials (host-bound, batch 2) and the ResNet bench: off / min 8M / min 32M / all.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s71
mkdir -p $O
export TMPDIR=/tmp
for m in fasterrcnn retinanet; do
  for cfg in "0 0" "1 8000000" "1 32000000" "1 0" "0 0" "1 8000000" "1 32000000" "1 0"; do
    set -- $cfg
    DET_WGRAD_STREAM=$1 DET_WGRAD_STREAM_MIN=$2 timeout -k 10 400 python -u scripts/bench_detection.py --model $m --amp O2 \
      --steps 30 --warmup 10 > $O/d.json 2> $O/d.err || { echo "$m $cfg failed rc=$?"; tail -8 $O/d.err; exit 1; }
    line=$(grep '^{' $O/d.json | tail -1)
    echo "{\"model\": \"$m\", \"side\": $1, \"min\": $2, \"bench\": $line}" >> $O/det.jsonl
    echo "$m side=$1 min=$2: $(echo "$line" | grep -o '"value": [0-9.]*')"
  done
done
for cfg in "1 0" "1 8000000" "1 32000000" "1 0" "1 8000000" "1 32000000"; do
  set -- $cfg
  DET_WGRAD_STREAM=$1 DET_WGRAD_STREAM_MIN=$2 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/b.json 2> $O/b.err \
    || { echo "bench $cfg rc=$?"; tail -20 $O/b.err; exit 1; }
  line=$(grep '^{' $O/b.json | tail -1)
  echo "{\"model\": \"resnet50\", \"side\": $1, \"min\": $2, \"bench\": $line}" >> $O/det.jsonl
  echo "resnet side=$1 min=$2: $(echo "$line" | grep -o '"value": [0-9.]*')"
done
