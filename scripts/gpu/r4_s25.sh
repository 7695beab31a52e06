#!/bin/bash
# Round-4 session 25: session 24 isolated the CIFAR hipGraph NaN to O2 + dropout (no NaN without
# dropout, none at O0 with dropout).  Does torch's dropout draw fresh masks under replays?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s25
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_graph_dropout_gpu.py > $O/test.log 2>&1; rc=$?
tail -15 $O/test.log
exit $rc
