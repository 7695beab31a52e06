#!/bin/bash
# Round-4 session 25: session 24 isolated the CIFAR hipGraph NaN to O2 + dropout (no NaN without
# dropout, none at O0 with dropout).  Does torch's dropout draw fresh masks under replays?  Then
# the graph GPU tests with the half-precision dropout guard, and the O2 CIFAR trial staying eager.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s25
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_graph_dropout_gpu.py > $O/test.log 2>&1
tail -12 $O/test.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_graph_gpu.py tests/test_graph_chunks.py tests/test_bert_trial_resume.py > $O/graph_tests.log 2>&1 || { tail -30 $O/graph_tests.log; exit 1; }
tail -3 $O/graph_tests.log
timeout -k 10 180 python -u scripts/bench_cifar_trial.py --batch 32 --batches 1000 --chunk 250 --amp O2 --lr 1e-4 --seed 1 \
  --hip-graph --graph-batches 20 > $O/cifar_o2_guard.json 2> $O/cifar_o2_guard.err || { tail -30 $O/cifar_o2_guard.err; exit 1; }
cat $O/cifar_o2_guard.json
