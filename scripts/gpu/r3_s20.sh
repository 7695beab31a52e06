#!/bin/bash
# Round-3 session 20: Mask R-CNN / RetinaNet fp32 at 2 images per GPU, default synthetic load vs the
# COCO-like instance load (mean 7.3 instances, heavy tail, small objects).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s20
mkdir -p $O
export TMPDIR=/tmp
for m in maskrcnn retinanet; do
  timeout -k 10 300 python -u scripts/bench_detection.py --model $m --steps 30 --warmup 10 --amp O0 > $O/${m}_O0.json 2> $O/${m}_O0.err || { tail -30 $O/${m}_O0.err; exit 1; }
  cat $O/${m}_O0.json
  timeout -k 10 300 python -u scripts/bench_detection.py --model $m --steps 30 --warmup 10 --amp O0 --coco-instances > $O/${m}_O0_coco.json 2> $O/${m}_O0_coco.err || { tail -30 $O/${m}_O0_coco.err; exit 1; }
  cat $O/${m}_O0_coco.json
done
