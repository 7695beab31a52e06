#!/bin/bash
# Round-2 session 12: HIP-graph replay of train_batch: numerics vs eager (GPU tests) and the CIFAR
# trial's per-batch cost eager vs graph.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s12
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/s12/pytest.log 2>&1 || { tail -40 gpurun_out/s12/pytest.log; exit 1; }
tail -3 gpurun_out/s12/pytest.log
for b in 16 32 64; do
  timeout -k 10 200 python -u scripts/bench_cifar_trial.py --batch $b --batches 3000 --hip-graph > gpurun_out/s12/cifar_graph_b$b.json 2> gpurun_out/s12/cifar_graph_b$b.err || { tail -20 gpurun_out/s12/cifar_graph_b$b.err; exit 1; }
  cat gpurun_out/s12/cifar_graph_b$b.json
done
