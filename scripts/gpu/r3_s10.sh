#!/bin/bash
# Round-3 session 10: ASHA O2 with hip_graph_batches 20 -- capture failing trials' logs (SIGSEGV on resume).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s10
mkdir -p $O
export TMPDIR=/tmp DET_BENCH_LOGDIR=$O
timeout -k 10 500 python -u scripts/bench_asha.py --slots 1 --timeout 450 > $O/asha_o2_gb16.json 2> $O/asha_o2_gb16.err || { tail -30 $O/asha_o2_gb16.err; exit 1; }
cat $O/asha_o2_gb16.json
