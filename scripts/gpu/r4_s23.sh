#!/bin/bash
# Round-4 session 23: locate the batch where the session-21 hipGraph-chunk runs go NaN (chunk 6 of
# 250 = batches 1500-1750, which holds the first epoch end at batch 1563): per-batch losses of
# 20-batch chunks with steps of 250 (steps split chunks) and of 260 (they do not), and of
# per-batch graphs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s23
mkdir -p $O
export TMPDIR=/tmp
for cfg in "g20_c250:--chunk 250 --hip-graph --graph-batches 20" "g20_c260:--chunk 260 --hip-graph --graph-batches 20" "g1_c250:--chunk 250 --hip-graph --graph-batches 1"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 180 python -u scripts/bench_cifar_trial.py --batch 32 --batches 1820 --amp O2 --lr 1e-4 --seed 1 \
    --batch-losses $args > $O/$name.json 2> $O/$name.err || { tail -30 $O/$name.err; exit 1; }
  python3 -c "
import json, math
d = json.load(open('$O/$name.json')); b = d['batch_losses']
i = next((k for k, x in enumerate(b) if not math.isfinite(x)), None)
print('$name', d['hip_graph'], 'first non-finite batch', i, 'losses', [round(x, 3) for x in b[(i or 1560) - 6:(i or 1560) + 3]])"
done
grep -i "warn\|hip_graph" $O/g20_c250.err | sort | uniq -c | head -20
