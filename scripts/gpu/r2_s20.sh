#!/bin/bash
# Round-2 session 20: host profile of the graph-replayed CIFAR train loop + GPU kernel time per batch.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s20
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/dbg/profile_train_loop.py > gpurun_out/s20/host_prof.txt 2>&1 || { tail -30 gpurun_out/s20/host_prof.txt; exit 1; }
head -3 gpurun_out/s20/host_prof.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s20/prof -o cifar -- python3 $GRAFT_REPO_ROOT/scripts/bench_cifar_trial.py --batch 32 --batches 600 --chunk 300 --hip-graph > $GRAFT_REPO_ROOT/gpurun_out/s20/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/s20/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && find gpurun_out/s20/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/s20/kernel_stats.csv \; && find gpurun_out/s20/prof -name "*kernel_trace.csv" -size +20M -delete; ls -la gpurun_out/s20
