#!/bin/bash
# Round-2 session 16: where trial construction time goes (cProfile on the GPU box).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s16
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/dbg/profile_trial_build.py > gpurun_out/s16/prof.txt 2>&1 || { tail -30 gpurun_out/s16/prof.txt; exit 1; }
head -5 gpurun_out/s16/prof.txt
