#!/bin/bash
# Round-2 session 18 (seed 1: graph+zygote+dynamo preload+seeded MIOpen cache, then eager A/B): ASHA trials/hr at the BASELINE shape (reference cifar10_pytorch/adaptive.yaml
# unchanged: 16 trials, 32 epochs x 50k records, validation every epoch) on the box's one slot,
# trial containers forked from the agent's warm zygote.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s18
export TMPDIR=/tmp DET_BENCH_LOGDIR=$GRAFT_REPO_ROOT/gpurun_out/s18
timeout -k 10 1080 python -u scripts/bench_asha.py --slots 1 --timeout 1040 > gpurun_out/s18/asha.json 2> gpurun_out/s18/asha.err || { tail -30 gpurun_out/s18/asha.err; tail -30 gpurun_out/s18/agent-0.log; exit 1; }
cat gpurun_out/s18/asha.json
timeout -k 10 1000 python -u scripts/bench_asha.py --slots 1 --timeout 960 --no-hip-graph > gpurun_out/s18/asha_eager.json 2> gpurun_out/s18/asha_eager.err || { tail -30 gpurun_out/s18/asha_eager.err; exit 1; }
cat gpurun_out/s18/asha_eager.json
