#!/bin/bash
# Round-4 session 14: the ResNet DP equivalence tests (2 ranks sharing the GPU over gloo; O0 at a
# stable learning rate) and the small-launch attribution probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s14
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread -p no:cacheprovider -m gpu tests/test_dp_resnet_gpu.py > $O/pytest_dp.log 2>&1 || { tail -60 $O/pytest_dp.log; exit 1; }
grep "dp-vs-single\|passed\|failed" $O/pytest_dp.log | tail -6
timeout -k 10 300 python -u scripts/probe_small_launches.py --steps 3 --warmup 3 > $O/small_launches.txt 2>&1 || { tail -20 $O/small_launches.txt; exit 1; }
head -40 $O/small_launches.txt
