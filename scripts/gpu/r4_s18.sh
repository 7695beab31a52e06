#!/bin/bash
# Round-4 session 18: CIFAR trial loss per 250-batch chunk at O2 eager, O2 + hipGraph chunks, O0 +
# hipGraph chunks (session 17 reported a NaN average loss after 3000 batches at O2 with graphs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s18
mkdir -p $O
export TMPDIR=/tmp
for cfg in "o2_eager:--amp O2" "o2_graph:--amp O2 --hip-graph --graph-batches 20" "o0_graph:--amp O0 --hip-graph --graph-batches 20"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python -u scripts/bench_cifar_trial.py --batch 32 --batches 3000 --chunk 250 $args > $O/cifar_$name.json 2> $O/cifar_$name.err || { tail -30 $O/cifar_$name.err; exit 1; }
  echo "$name $(python3 -c "import json;d=json.load(open('$O/cifar_$name.json'));print(d['value'], d['validation_error'], [round(x,3) if x==x else x for x in d['loss_per_chunk']])")"
done
