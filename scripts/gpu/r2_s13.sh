#!/bin/bash
# Round-2 session 13: hipGraph capture probe (MLP, conv without MIOpen, conv with MIOpen), stops
# at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s13
export TMPDIR=/tmp
for c in mlp conv_native conv_miopen; do
  timeout -k 10 120 python -u scripts/dbg/graph_probe.py $c > gpurun_out/s13/$c.log 2>&1 || { echo "FAILED $c rc=$?"; tail -30 gpurun_out/s13/$c.log; exit 1; }
  tail -1 gpurun_out/s13/$c.log
done
