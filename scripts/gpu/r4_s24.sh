#!/bin/bash
# Round-4 session 24: the hipGraph NaN of session 23 comes at a random late batch (1355-1777) with
# per-batch graphs and with 20-batch chunks alike, never eagerly.  Which ingredient: dropout (torch
# Philox state under replays) or bf16 (O2)?  1820 batches, seed 1, lr 1e-4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s24
mkdir -p $O
export TMPDIR=/tmp
for cfg in "O2_g1_nodrop:--amp O2 --no-dropout --hip-graph --graph-batches 1" "O2_g20_nodrop:--amp O2 --no-dropout --hip-graph --graph-batches 20" "O0_g1_drop:--amp O0 --hip-graph --graph-batches 1" "O2_eager_drop:--amp O2"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 1820 --chunk 250 --lr 1e-4 --seed 1 \
    --batch-losses $args > $O/$name.json 2> $O/$name.err || { tail -30 $O/$name.err; exit 1; }
  python3 -c "
import json, math
d = json.load(open('$O/$name.json')); b = d['batch_losses']
i = next((k for k, x in enumerate(b) if not math.isfinite(x)), None)
print('$name', 'first non-finite batch', i, 'last', [round(x, 3) for x in b[-4:]], 'ms/batch', d['value'])"
done
