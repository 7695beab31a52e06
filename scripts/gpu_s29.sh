#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -q --timeout 200 --timeout-method thread 2>&1 | tail -2
timeout -k 10 200 python scripts/bench_attn.py 2>&1 | grep -v amdgpu.ids
