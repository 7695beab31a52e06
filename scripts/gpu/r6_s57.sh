#!/bin/bash
# Round-6 session 57: does the bench's linear-scaling learning rate stay finite at the 8-GPU global
# batch (8 x 1,024 -> lr 3.2)?  One GPU, lr 3.2 and 1.6, 60 timed steps: final loss and throughput.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s57
mkdir -p $O
export TMPDIR=/tmp
for lr in 3.2 1.6 0.4; do
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --lr $lr > $O/b.json 2> $O/b.err \
    || { echo "bench lr=$lr rc=$?"; tail -20 $O/b.err; exit 1; }
  line=$(grep '^{' $O/b.json | tail -1)
  echo "{\"lr\": $lr, \"bench\": $line}" >> $O/lr.jsonl
  echo "lr=$lr: $(echo "$line" | grep -o '"value": [0-9.]*\|"final_avg_loss": [^,]*' | tr '\n' ' ')"
done
