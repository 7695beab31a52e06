#!/bin/bash
# Round-3 session 5: per-shape 3x3 conv pass timing native vs MIOpen (fwd / dgrad / wgrad).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3s5
export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/bench_conv3x3.py 512 > gpurun_out/r3s5/conv3x3.jsonl 2> gpurun_out/r3s5/conv3x3.err || { tail -20 gpurun_out/r3s5/conv3x3.err; exit 1; }
cat gpurun_out/r3s5/conv3x3.jsonl
