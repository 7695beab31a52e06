#!/bin/bash
# Session: ResNet-50 conv shapes — MIOpen (find mode) vs hipBLASLt GEMM for 1x1 convs.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/microbench_conv.py 1 512 > gpurun_out/conv_mb.log 2>&1
echo "rc=$?"
cat gpurun_out/conv_mb.log | grep -v amdgpu.ids
