#!/bin/bash
# Round-6 session 49: per-GPU batch sweep of the default (eager + side-stream weight gradients)
# step: 512 / 768 / 1024, two alternating passes.  (r6 graph-mode sweep:
# profiles/r6_bench_resnet50_batch_sweep.jsonl, 12,631 / 12,735 / 12,928.)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s49
mkdir -p $O
export TMPDIR=/tmp
BS_LIST=${BS_LIST:-512 768 1024}
for rep in 1 2; do
  for bs in $BS_LIST; do
    timeout -k 10 400 python -u bench.py --steps 40 --warmup 10 --batch-per-gpu $bs > $O/b.json 2> $O/b.err \
      || { echo "bench bs=$bs rc=$?"; tail -20 $O/b.err; exit 1; }
    grep '^{' $O/b.json | tail -1 >> $O/sweep.jsonl
    echo "bs=$bs rep=$rep: $(grep '^{' $O/b.json | tail -1 | cut -c60-140)"
  done
done
