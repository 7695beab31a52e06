#!/bin/bash
# Round-5 session 29: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) for the launch-bound
# CIFAR trial and the BERT step; ResNet bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s29
mkdir -p $O
export TMPDIR=/tmp
for k in 0 1 0 1; do
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 \
    --amp O2 --hip-graph --graph-batches 20 --lr 1e-4 > $O/cifar.json 2> $O/cifar.err || { tail -20 $O/cifar.err; exit 1; }
  echo "kernarg=$k cifar O2: $(grep -o '"value": [0-9.]*' $O/cifar.json)" | tee -a $O/ab.txt
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 300 python -u scripts/bench_bert.py --steps 60 --warmup 8 > $O/bert.json 2> $O/bert.err || { tail -12 $O/bert.err; exit 1; }
  echo "kernarg=$k bert eager: $(grep -o '"value": [0-9.]*' $O/bert.json)" | tee -a $O/ab.txt
done
for k in 0 1; do
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo "kernarg=$k resnet bench: $(grep -o '"value": [0-9.]*' $O/bench.json)" | tee -a $O/ab.txt
done
