#!/bin/bash
# Round-4 session 21: is the NaN of session 18 (O2 + 20-batch hipGraph chunks, lr 1e-3, 3000
# batches) a property of the run or of the graph path?  O2 eager and O2 graph chunks at seeds 1-3,
# lr 1e-3 (the bench's) and 1e-4 (the reference const.yaml's), loss per 250-batch chunk.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s21
mkdir -p $O
export TMPDIR=/tmp
for lr in 1e-3 1e-4; do
  for seed in 1 2 3; do
    for cfg in "eager:" "g20:--hip-graph --graph-batches 20"; do
      name=lr${lr}_s${seed}_${cfg%%:*}; args=${cfg#*:}
      timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 3000 --chunk 250 --amp O2 \
        --lr $lr --seed $seed $args > $O/$name.json 2> $O/$name.err || { tail -30 $O/$name.err; exit 1; }
      echo "$name $(python3 -c "import json;d=json.load(open('$O/$name.json'));print(d['validation_error'], [round(x,3) if x==x else x for x in d['loss_per_chunk']])")"
    done
  done
done
