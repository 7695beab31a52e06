#!/bin/bash
# Round-2 session 19: CIFAR trial with uint8 batches + GPU normalize (graph replay): per-batch cost,
# then ASHA at the reference adaptive.yaml shape (seed 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s19
export TMPDIR=/tmp DET_BENCH_LOGDIR=$GRAFT_REPO_ROOT/gpurun_out/s19
for b in 16 32 64; do
  timeout -k 10 200 python -u scripts/bench_cifar_trial.py --batch $b --batches 3000 --hip-graph > gpurun_out/s19/cifar_graph_b$b.json 2> gpurun_out/s19/cifar_graph_b$b.err || { tail -20 gpurun_out/s19/cifar_graph_b$b.err; exit 1; }
  cat gpurun_out/s19/cifar_graph_b$b.json
done
timeout -k 10 900 python -u scripts/bench_asha.py --slots 1 --timeout 860 > gpurun_out/s19/asha.json 2> gpurun_out/s19/asha.err || { tail -30 gpurun_out/s19/asha.err; exit 1; }
cat gpurun_out/s19/asha.json
