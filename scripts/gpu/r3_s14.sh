#!/bin/bash
# Round-3 session 14: det_igemm_wgrad with multi-group stages + split-lane slab reduce: numerics, microbench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s14
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py -k "ring_wgrad" > $O/pytest_wgrad.log 2>&1 || { tail -40 $O/pytest_wgrad.log; exit 1; }
tail -2 $O/pytest_wgrad.log
timeout -k 10 500 python -u scripts/bench_wgrad.py > $O/wgrad.jsonl 2> $O/wgrad.err || { tail -20 $O/wgrad.err; exit 1; }
tail -1 $O/wgrad.jsonl
