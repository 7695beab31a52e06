#!/bin/bash
# Round-2 session 14: bisect the capture_end segfault (probe variants first, controller last).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s14
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
i=0
for args in "conv_miopen --maxpool" "conv_miopen --maxpool --bench"; do
  i=$((i+1))
  timeout -k 10 120 python -u scripts/dbg/graph_probe.py $args > gpurun_out/s14/p$i.log 2>&1 || { echo "FAILED $args"; tail -30 gpurun_out/s14/p$i.log; exit 1; }
  tail -1 gpurun_out/s14/p$i.log
done
DET_GRAD_SINK=0 timeout -k 10 120 python -u scripts/dbg/graph_ctrl_probe.py > gpurun_out/s14/ctrl_nosink.log 2>&1 || { echo "FAILED ctrl nosink"; grep -v "^  File \"/usr" gpurun_out/s14/ctrl_nosink.log | tail -30; exit 1; }
tail -1 gpurun_out/s14/ctrl_nosink.log
