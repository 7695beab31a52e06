#!/bin/bash
# Round-6 session 26: det_gemm8 (eight-phase 256x256 GEMM) numerics, then timing vs hipBLASLt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s26; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm8_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|error" $O/test.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_gemm8.py > $O/bench.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.jsonl
