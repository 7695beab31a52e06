#!/bin/bash
# Round-5 session 36: stacked metrics straight to host (one concat + copy per step / validation):
# graph tests, CIFAR trial with repeated validations, ASHA O0 twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s36
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py tests/test_graph_cifar_o2_gpu.py tests/test_cnn_gpu.py tests/test_examples_gpu.py \
  -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 100 --amp O0 --hip-graph \
  --graph-batches 20 --lr 1e-4 --validations 6 > $O/cifar_val.json 2> $O/cifar.err || { tail -20 $O/cifar.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/cifar_val.json')); print('O0 chunk100', d['value'], d['validation_10k_s'], d['validation_10k_s_later'])"
for i in 1 2; do
  DET_BENCH_LOGDIR=$O timeout -k 10 600 python -u scripts/bench_asha.py --slots 1 --amp O0 --graph-batches 20 --timeout 540 \
    > $O/asha_O0_$i.json 2> $O/asha_O0.err || { echo "asha O0 rc=$?"; tail -20 $O/asha_O0.err; exit 1; }
  echo "asha O0 #$i: $(grep '^{' $O/asha_O0_$i.json | tail -1 | cut -c1-200)"
done
