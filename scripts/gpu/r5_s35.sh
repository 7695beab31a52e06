#!/bin/bash
# Round-5 session 35: CIFAR validation cost (first pass captures, later ones replay) and its host
# profile, O0 as in the ASHA benchmark.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s35
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 1000 --chunk 500 --amp O0 --hip-graph \
  --graph-batches 20 --lr 1e-4 --validations 6 > $O/cifar_val.json 2> $O/cifar.err || { tail -20 $O/cifar.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/cifar_val.json')); print(d['value'], d['validation_10k_s'], d['validation_10k_s_later'])"
timeout -k 10 240 python -u -m cProfile -o $O/cifar_val.cprof scripts/bench_cifar_trial.py --batch 32 --batches 500 --chunk 500 \
  --amp O0 --hip-graph --graph-batches 20 --lr 1e-4 --validations 21 > $O/cifar_val_cprof.json 2> $O/cifar.err || { tail -20 $O/cifar.err; exit 1; }
python3 scripts/cprof_summary.py $O/cifar_val.cprof 45 > $O/cifar_val_cprof.txt 2>&1
python3 -c "import json; d=json.load(open('$O/cifar_val_cprof.json')); print(d['validation_10k_s_later'])"
