#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 120 python scripts/dbg_pool.py 2>&1 | grep -v amdgpu.ids
