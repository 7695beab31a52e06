#!/bin/bash
# Round-6 session 53: training step on a high-priority stream (DET_COMPUTE_STREAM_HIGH_PRIO=1) so the
# side-stream weight gradients yield to the input-gradient chain; A/B at 1,024 and 512 images/GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s53
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for bs in 1024 512; do
    for hp in 0 1; do
      DET_COMPUTE_STREAM_HIGH_PRIO=$hp timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --batch-per-gpu $bs \
        > $O/b.json 2> $O/b.err || { echo "bench hp=$hp bs=$bs rc=$?"; tail -20 $O/b.err; exit 1; }
      line=$(grep '^{' $O/b.json | tail -1)
      echo "{\"high_prio\": $hp, \"bs\": $bs, \"bench\": $line}" >> $O/ab.jsonl
      echo "hp=$hp bs=$bs: $(echo "$line" | cut -c60-110)"
    done
  done
done
