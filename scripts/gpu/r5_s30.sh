#!/bin/bash
# Round-5 session 30: ResNet-50 bench with kernel arguments in device memory, alternating A/B x3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s30
mkdir -p $O
export TMPDIR=/tmp
for k in 1 0 1 0 1 0; do
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo "{\"HIP_FORCE_DEV_KERNARG\": $k, \"result\": $(grep '^{' $O/bench.json | tail -1)}" >> $O/kernarg_ab.jsonl
  echo "kernarg=$k resnet bench: $(grep -o '"value": [0-9.]*' $O/bench.json)"
done
