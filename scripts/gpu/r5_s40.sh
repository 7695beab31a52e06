#!/bin/bash
# Round-5 session 40 (final): the whole GPU suite + smoke(), then the headline numbers once more --
# bench.py (ResNet-50), BERT eager / hipGraph, CIFAR trial O2 / O0, ASHA O0.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s40
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.log 2>&1
rc=$?; tail -3 $O/gpu_suite.log; grep -E "FAILED|ERROR" $O/gpu_suite.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench: $(cut -c1-200 $O/bench.json)"
for g in "" "--hip-graph"; do
  timeout -k 10 300 python -u scripts/bench_bert.py --steps 60 --warmup 8 $g > $O/bert$g.json 2> $O/bert.err || { tail -12 $O/bert.err; exit 1; }
  echo "bert $g: $(grep -o '"value": [0-9.]*' $O/bert$g.json)"
done
for amp in O2 O0; do
  timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 \
    --amp $amp --hip-graph --graph-batches 20 --lr 1e-4 > $O/cifar_$amp.json 2> $O/cifar.err || { tail -20 $O/cifar.err; exit 1; }
  echo "cifar $amp: $(grep -o '"value": [0-9.]*' $O/cifar_$amp.json)"
done
DET_BENCH_LOGDIR=$O timeout -k 10 600 python -u scripts/bench_asha.py --slots 1 --amp O0 --graph-batches 20 --timeout 540 \
  > $O/asha_O0.json 2> $O/asha_O0.err || { echo "asha O0 rc=$?"; tail -20 $O/asha_O0.err; exit 1; }
echo "asha O0: $(grep '^{' $O/asha_O0.json | tail -1 | cut -c1-160)"
