#!/bin/bash
# Round-6 session 68: the data-parallel path of the driver's scaling run at full size on one GPU:
# bench.py defaults (1,024 images, eager + side-stream weight gradients) with a world-1 RCCL group
# (DET_FORCE_DISTRIBUTED=1: bucketed fp32-accumulate all-to-all + sum + all-gather overlapped with
# backward, GradSink flush joins) and the phase timers the multi-GPU runs keep on; vs the plain run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s68
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + rep)) \
    DET_FORCE_DISTRIBUTED=1 DET_STEP_TIMERS=1 timeout -k 10 400 python -u bench.py --steps 30 --warmup 10 \
    > $O/dp.json 2> $O/dp.err || { echo "dp rc=$?"; tail -30 $O/dp.err; exit 1; }
  line=$(grep '^{' $O/dp.json | tail -1)
  echo "{\"mode\": \"dp_world1_rccl\", \"bench\": $line}" >> $O/dp.jsonl
  echo "dp: $(echo "$line" | grep -o '"value": [0-9.]*\|"backend": "[a-z]*"\|"phase_ms": {[^}]*}\|"final_avg_loss": [0-9.]*' | tr '\n' ' ')"
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/b.json 2> $O/b.err || { echo "plain rc=$?"; tail -20 $O/b.err; exit 1; }
  line=$(grep '^{' $O/b.json | tail -1)
  echo "{\"mode\": \"plain\", \"bench\": $line}" >> $O/dp.jsonl
  echo "plain: $(echo "$line" | grep -o '"value": [0-9.]*\|"final_avg_loss": [0-9.]*' | tr '\n' ' ')"
done
