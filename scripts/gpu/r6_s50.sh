#!/bin/bash
# Round-6 session 50: bench.py with the new defaults (per-GPU batch 1024, eager + side-stream
# weight gradients) three times, as the driver runs it (no flags).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s50
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py > $O/b.json 2> $O/b.err || { echo "bench rc=$?"; tail -20 $O/b.err; exit 1; }
  grep '^{' $O/b.json | tail -1 >> $O/defaults.jsonl
  echo "run $i: $(grep '^{' $O/b.json | tail -1 | cut -c60-140)"
done
