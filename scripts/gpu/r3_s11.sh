#!/bin/bash
# Round-3 session 11: CIFAR trial ms/batch (bs 32 / 64) per-batch graph vs 20-batch graphs, and a
# kernel-trace of the chunked run (GPU time per batch).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s11
mkdir -p $O
export TMPDIR=/tmp
for b in 32 64; do
  timeout -k 10 200 python -u scripts/bench_cifar_trial.py --batch $b --batches 3000 --chunk 100 --hip-graph > $O/cifar_b${b}_g1.json 2> $O/cifar_b${b}_g1.err || { tail -20 $O/cifar_b${b}_g1.err; exit 1; }
  cat $O/cifar_b${b}_g1.json
  timeout -k 10 200 python -u scripts/bench_cifar_trial.py --batch $b --batches 3000 --chunk 100 --hip-graph --graph-batches 20 > $O/cifar_b${b}_g20.json 2> $O/cifar_b${b}_g20.err || { tail -20 $O/cifar_b${b}_g20.err; exit 1; }
  cat $O/cifar_b${b}_g20.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u scripts/bench_cifar_trial.py --batch 64 --batches 3000 --chunk 100 --hip-graph --graph-batches 20 > $O/prof_run.json 2> $O/prof_run.err || { tail -20 $O/prof_run.err; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
cp "$f" $O/cifar_b64_g20_kernel_stats.csv
head -30 $O/cifar_b64_g20_kernel_stats.csv
rm -rf $O/prof
