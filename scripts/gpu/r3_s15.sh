#!/bin/bash
# Round-3 session 15: det_igemm_wgrad split rule (>= one wave of workgroups): numerics + microbench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s15
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py -k "ring_wgrad" > $O/pytest_wgrad.log 2>&1 || { tail -40 $O/pytest_wgrad.log; exit 1; }
tail -2 $O/pytest_wgrad.log
timeout -k 10 500 python -u scripts/bench_wgrad.py --cfgs 1,2,3,4,5,6,7,9,10 > $O/wgrad.jsonl 2> $O/wgrad.err || { tail -20 $O/wgrad.err; exit 1; }
tail -1 $O/wgrad.jsonl
