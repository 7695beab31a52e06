#!/bin/bash
# Round-2 session 22: RCCL kernel trace of a ResNet-50 data-parallel step (world 1 over nccl,
# forced distributed: bucketed all-to-all + fp32 shard sum + all-gather on RCCL's stream) and its
# overlap with backward compute.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s22
export TMPDIR=/tmp
export DET_FORCE_DISTRIBUTED=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/s22/prof -o dp -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/s22/bench.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/s22/bench.log; exit 1; }
cd $GRAFT_REPO_ROOT && grep '^{"metric"' gpurun_out/s22/bench.log | tail -1
python scripts/dbg/rccl_overlap.py gpurun_out/s22/prof/dp_results.db > gpurun_out/s22/rccl_overlap.txt && cat gpurun_out/s22/rccl_overlap.txt
python scripts/dbg/rocpd_summary.py gpurun_out/s22/prof/dp_results.db 40 > gpurun_out/s22/kernels.txt && rm -rf gpurun_out/s22/prof
