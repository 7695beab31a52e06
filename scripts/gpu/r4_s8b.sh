#!/bin/bash
# Round-4 session 8b: the affine-residual (deferred shortcut BN) kernels in isolation and in a block.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s8b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_bn_bwd_fusion_gpu.py -k "affine or projection_shortcut_bn_apply" > $O/pytest.log 2>&1; tail -40 $O/pytest.log | grep -v "^$"
