#!/bin/bash
# Round-5 session 41: CNN dropout drawn in the epilogues (no mask kernel / tensors): CNN + graph
# tests, CIFAR O2/O0.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s41
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py tests/test_graph_cifar_o2_gpu.py tests/test_examples_gpu.py -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for amp in O2 O0 O2 O0; do
  timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 \
    --amp $amp --hip-graph --graph-batches 20 --lr 1e-4 > $O/cifar_$amp.json 2> $O/cifar.err || { tail -20 $O/cifar.err; exit 1; }
  echo "cifar $amp: $(cut -c1-100 $O/cifar_$amp.json) loss $(grep -o '"loss": [0-9.]*' $O/cifar_$amp.json)"; cat $O/cifar_$amp.json >> $O/cifar_runs.jsonl
done
