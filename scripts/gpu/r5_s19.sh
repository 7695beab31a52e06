#!/bin/bash
# Round-5 session 19: CIFAR split-K sizing A/B (DET_CNN_BLOCKS) without the metric-gradient fills;
# then ASHA trials/hr at the reference adaptive.yaml shape, O0 and O2, 1 GPU slot.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s19
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py -q --timeout 300 --timeout-method thread > $O/cnn_tests.log 2>&1 || { tail -30 $O/cnn_tests.log; exit 1; }
tail -1 $O/cnn_tests.log
for b in 1024 512 768 384; do
  DET_CNN_BLOCKS=$b timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 \
    --amp O2 --hip-graph --graph-batches 20 --lr 1e-4 > $O/cifar_b$b.json 2> $O/cifar.err || { tail -20 $O/cifar.err; exit 1; }
  echo "blocks $b: $(cut -c1-120 $O/cifar_b$b.json)"
done
for amp in O0 O2; do
  DET_BENCH_LOGDIR=$O timeout -k 10 900 python -u scripts/bench_asha.py --slots 1 --amp $amp --graph-batches 20 --timeout 840 \
    > $O/asha_$amp.json 2> $O/asha_$amp.err || { echo "asha $amp rc=$?"; tail -20 $O/asha_$amp.err; exit 1; }
  echo "asha $amp: $(grep '^{' $O/asha_$amp.json | tail -1 | cut -c1-700)"
done
