#!/bin/bash
# Round-2 session 2: in-tree seeded MIOpen db on a fresh box; immediate-mode A/B; forced-distributed
# (world 1, RCCL) bench under rocprofv3 showing the all-to-all / all-gather / det_sum_rows path.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s2
export TMPDIR=/tmp
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s2/bench_seeded.json 2> gpurun_out/s2/bench_seeded.err || { tail -20 gpurun_out/s2/bench_seeded.err; exit 1; }
cat gpurun_out/s2/bench_seeded.json
MIOPEN_USER_DB_PATH=$PWD/gpurun_out/s2/imm_db MIOPEN_CUSTOM_CACHE_DIR=$PWD/gpurun_out/s2/imm_cache \
  timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 --cudnn-benchmark 0 > gpurun_out/s2/bench_immediate.json 2> gpurun_out/s2/bench_immediate.err || { tail -20 gpurun_out/s2/bench_immediate.err; exit 1; }
cat gpurun_out/s2/bench_immediate.json
export DET_FORCE_DISTRIBUTED=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d gpurun_out/s2/prof_dist -o run -- python3 -u bench.py --steps 10 --warmup 5 > gpurun_out/s2/bench_dist1.json 2> gpurun_out/s2/bench_dist1.err || { tail -20 gpurun_out/s2/bench_dist1.err; exit 1; }
cat gpurun_out/s2/bench_dist1.json
find gpurun_out/s2/prof_dist -name "*stats*" | head
