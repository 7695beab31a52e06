#!/bin/bash
# Round-6 session 66: CIFAR trial per-batch cost at O0 vs the hipGraph chunk length (batches per
# replay: 20 / 50 / 100).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s66
mkdir -p $O
export TMPDIR=/tmp
for gb in 20 50 100 20; do
  timeout -k 10 300 python -u scripts/bench_cifar_trial.py --batch 32 --batches 3000 --amp O0 --hip-graph --graph-batches $gb \
    > $O/c.json 2> $O/c.err || { echo "cifar gb=$gb rc=$?"; tail -20 $O/c.err; exit 1; }
  line=$(grep '^{' $O/c.json | tail -1)
  echo "{\"graph_batches\": $gb, \"bench\": $line}" >> $O/gb.jsonl
  echo "gb=$gb: $(echo "$line" | grep -o '"value": [0-9.]*')"
done
