#!/bin/bash
# Round-6 session 54: side stream on a CU mask (DET_WGRAD_STREAM_RESERVE=k leaves every k-th CU to the
# main stream); bench at 1,024 images/GPU, k = 0 (all CUs) / 16 / 8 / 4, two passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s54
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for k in 0 16 8 4; do
    DET_WGRAD_STREAM_RESERVE=$k timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/b.json 2> $O/b.err \
      || { echo "bench k=$k rc=$?"; tail -20 $O/b.err; exit 1; }
    line=$(grep '^{' $O/b.json | tail -1)
    echo "{\"reserve\": $k, \"bench\": $line}" >> $O/ab.jsonl
    echo "k=$k: $(echo "$line" | cut -c60-110)"
  done
done
