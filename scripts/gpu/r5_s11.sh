#!/bin/bash
# Round-5 session 11: (a) native CIFAR CNN with split-K everywhere (pooled convs finished by the
# finish kernel); (b) MIOpen graph divergence: per-op with eager calls interleaved, 1- and 2-step
# graphs, fp16.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s11
mkdir -p $O
export TMPDIR=/tmp
R="python -u scripts/dbg/miopen_graph_repro.py"
timeout -k 10 300 $R --k 20 --replays 3 --interleave > $O/ops_inter.log 2>&1 || { echo "ops rc=$?"; tail -20 $O/ops_inter.log; exit 1; }
echo "== ops interleaved"; grep -E '"op"|"bad"' $O/ops_inter.log | cut -c1-200
for cfg in "k1:--step --k 1 --replays 30 --arch conv" "k2:--step --k 2 --replays 15 --arch conv" "fp16:--step --k 20 --replays 4 --arch conv --dtype fp16"; do
  name=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 300 $R $a > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "== $name"; grep -E '"mode"' $O/$name.log | cut -c1-150 | awk 'NR<=6 || /false/' | head -12
done
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py tests/test_graph_dropout_gpu.py -v --timeout 120 --timeout-method thread > $O/cnn_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/cnn_tests.log | head -30
[ $rc -le 1 ] || { tail -c 3000 $O/cnn_tests.log; exit $rc; }
[ $rc -eq 0 ] || { grep -E "^E  " $O/cnn_tests.log | grep -v "tensor(" | head -20; exit 1; }
for amp in O2 O0; do
  DET_GRAPH_HALF_DROPOUT=1 timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 \
    --amp $amp --hip-graph --graph-batches 20 --lr 1e-4 > $O/cifar_$amp.json 2> $O/cifar_$amp.err
  rc=$?; echo "cifar $amp rc=$rc: $(cut -c1-300 $O/cifar_$amp.json)"
  [ $rc -le 1 ] || { tail -30 $O/cifar_$amp.err; exit $rc; }
done
DET_GRAPH_HALF_DROPOUT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o cifar -- \
  python3 -u scripts/bench_cifar_trial.py --batch 32 --batches 1000 --chunk 500 --amp O2 --hip-graph --graph-batches 20 \
  --lr 1e-4 > $O/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $O/prof.log; exit 1; }
echo "prof done"
