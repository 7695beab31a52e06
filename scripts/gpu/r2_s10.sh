#!/bin/bash
# Round-2 session 10: per-batch cost of the ASHA benchmark's CIFAR-10 trial (batch 16/32/64) and a
# kernel-trace profile of the batch-32 run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s10
export TMPDIR=/tmp
for b in 16 32 64; do
  timeout -k 10 200 python -u scripts/bench_cifar_trial.py --batch $b --batches 3000 > gpurun_out/s10/cifar_b$b.json 2> gpurun_out/s10/cifar_b$b.err || { tail -20 gpurun_out/s10/cifar_b$b.err; exit 1; }
  cat gpurun_out/s10/cifar_b$b.json
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s10/prof -o cifar -- python3 $GRAFT_REPO_ROOT/scripts/bench_cifar_trial.py --batch 32 --batches 2000 > $GRAFT_REPO_ROOT/gpurun_out/s10/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/s10/prof.log; exit 1; }
tail -2 $GRAFT_REPO_ROOT/gpurun_out/s10/prof.log
