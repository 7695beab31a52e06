#!/bin/bash
# Round-2 session 6: pipelined implicit-GEMM conv (det_igemm) numerics + ResNet-50 conv microbench;
# the fp32 shortcut-link BN test in isolation (flaked once in s5).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s6
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_igemm_gpu.py > gpurun_out/s6/pytest_igemm.log 2>&1; rc=$?
tail -15 gpurun_out/s6/pytest_igemm.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u scripts/bench_igemm.py 512 > gpurun_out/s6/igemm.jsonl 2> gpurun_out/s6/igemm.err || { tail -20 gpurun_out/s6/igemm.err; exit 1; }
cat gpurun_out/s6/igemm.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread "tests/test_norm_gpu.py::test_resnet50_fused_shortcut_link_and_pool_match_stock" tests/test_norm_gpu.py > gpurun_out/s6/pytest_norm.log 2>&1; rc2=$?
tail -5 gpurun_out/s6/pytest_norm.log
exit $rc
