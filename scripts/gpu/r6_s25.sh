#!/bin/bash
# Round-6 session 25: Mask R-CNN native vs MIOpen convolutions, alternating order (order effects of
# r6s24: the first run of each pair was the slower one).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s25; mkdir -p $O
export TMPDIR=/tmp
for amp in O2 O0; do
  for nc in 0 1 0 1; do
    i=$((i+1))
    DET_NATIVE_CONV2D=$nc timeout -k 10 400 python -u scripts/bench_detection.py --model maskrcnn --amp $amp --steps 30 --warmup 10 > $O/maskrcnn_${amp}_nc${nc}_$i.json 2> $O/maskrcnn_${amp}_nc${nc}_$i.err || { echo "failed"; tail -8 $O/maskrcnn_${amp}_nc${nc}_$i.err; exit 1; }
    echo "maskrcnn $amp native=$nc run $i: $(tail -1 $O/maskrcnn_${amp}_nc${nc}_$i.json | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["config"].get("s_per_iter"), d["config"].get("native_conv2d"))')"
  done
done
