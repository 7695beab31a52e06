#!/bin/bash
# Round-2 session 17: seed the MIOpen db + kernel cache for the CIFAR trial's batch sizes 16..64
# and harvest it (copied into determined_1_amd/ops/miopen_db afterwards).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s17
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/miopen_seed_cifar.py --harvest gpurun_out/s17/miopen_db > gpurun_out/s17/seed.log 2>&1 || { tail -30 gpurun_out/s17/seed.log; exit 1; }
tail -5 gpurun_out/s17/seed.log
ls -la gpurun_out/s17/miopen_db/*
