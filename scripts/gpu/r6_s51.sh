#!/bin/bash
# Round-6 session 51: CIFAR-10 trial (ASHA benchmark) per-batch cost on the round-6 tree, O0 / O2,
# batch 32, 20-batch graph chunks, and a kernel trace of the O0 run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s51
mkdir -p $O
export TMPDIR=/tmp
for amp in O0 O2 O0; do
  timeout -k 10 300 python -u scripts/bench_cifar_trial.py --batch 32 --batches 3000 --amp $amp --hip-graph --graph-batches 20 \
    > $O/c.json 2> $O/c.err || { echo "cifar $amp rc=$?"; tail -20 $O/c.err; exit 1; }
  grep '^{' $O/c.json | tail -1 >> $O/cifar.jsonl
  echo "$amp: $(grep '^{' $O/c.json | tail -1 | cut -c1-300)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o cifar -- python3 -u scripts/bench_cifar_trial.py --batch 32 \
  --batches 2000 --amp O0 --hip-graph --graph-batches 20 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
