#!/bin/bash
# Round-2 session 8: ALBERT-xxlarge SQuAD at the reference const.yaml config (fp32 = amp O0,
# batch 2, aggregation_frequency 24) for a like-for-like examples/s vs the published 2.0 (V100),
# plus the same batch/aggregation in bf16 O2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s8
export TMPDIR=/tmp
timeout -k 10 560 python -u scripts/bench_albert.py --amp O0 --batch-per-gpu 2 --agg 24 --steps 3 --warmup 1 > gpurun_out/s8/albert_fp32.json 2> gpurun_out/s8/albert_fp32.err || { tail -20 gpurun_out/s8/albert_fp32.err; exit 1; }
cat gpurun_out/s8/albert_fp32.json
timeout -k 10 400 python -u scripts/bench_albert.py --amp O2 --batch-per-gpu 2 --agg 24 --steps 3 --warmup 1 > gpurun_out/s8/albert_bf16_b2.json 2> gpurun_out/s8/albert_bf16_b2.err || { tail -20 gpurun_out/s8/albert_bf16_b2.err; exit 1; }
cat gpurun_out/s8/albert_bf16_b2.json
