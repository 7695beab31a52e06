#!/bin/bash
# Round-2 session 21: eval-graph GPU test, channels_last CIFAR trial per-batch cost + kernel census,
# ASHA at the reference shape (seed 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s21
export TMPDIR=/tmp DET_BENCH_LOGDIR=$GRAFT_REPO_ROOT/gpurun_out/s21
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/s21/pytest.log 2>&1 || { tail -40 gpurun_out/s21/pytest.log; exit 1; }
tail -2 gpurun_out/s21/pytest.log
for b in 16 32 64; do
  timeout -k 10 200 python -u scripts/bench_cifar_trial.py --batch $b --batches 3000 --hip-graph > gpurun_out/s21/cifar_b$b.json 2> gpurun_out/s21/cifar_b$b.err || { tail -20 gpurun_out/s21/cifar_b$b.err; exit 1; }
  cat gpurun_out/s21/cifar_b$b.json
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/s21/prof -o cifar -- python3 $GRAFT_REPO_ROOT/scripts/bench_cifar_trial.py --batch 32 --batches 600 --chunk 300 --hip-graph > $GRAFT_REPO_ROOT/gpurun_out/s21/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/s21/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/dbg/rocpd_summary.py gpurun_out/s21/prof/cifar_results.db 30 > gpurun_out/s21/kernels.txt && rm -rf gpurun_out/s21/prof && head -12 gpurun_out/s21/kernels.txt
timeout -k 10 900 python -u scripts/bench_asha.py --slots 1 --timeout 860 > gpurun_out/s21/asha.json 2> gpurun_out/s21/asha.err || { tail -30 gpurun_out/s21/asha.err; exit 1; }
cat gpurun_out/s21/asha.json
