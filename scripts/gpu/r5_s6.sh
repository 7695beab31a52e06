#!/bin/bash
# Round-5 session 6: (a) native CIFAR CNN tests after the 32-bit / vector gather-loader rewrite and the
# CIFAR trial speed (O2, O0) plus a kernel trace of it; (b) chunk-graph replay vs per-batch replay vs
# eager from one state on the same batches (bank masks / no dropout / torch dropout); (c) the O2
# chunked-graph NaN with per-chunk checks: separate pools, O0, no dropout, bank masks, native CNN.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s6
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py -v --timeout 120 --timeout-method thread > $O/cnn_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/cnn_tests.log | head -20
[ $rc -le 1 ] || { tail -c 3000 $O/cnn_tests.log; exit $rc; }
[ $rc -eq 0 ] || grep -E "^E  " $O/cnn_tests.log | grep -v "tensor(" | head -20
for amp in O2 O0; do
  DET_GRAPH_HALF_DROPOUT=1 timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 \
    --amp $amp --hip-graph --graph-batches 20 --lr 1e-4 > $O/cifar_$amp.json 2> $O/cifar_$amp.err
  rc=$?; echo "cifar $amp rc=$rc: $(cut -c1-420 $O/cifar_$amp.json)"
  [ $rc -le 1 ] || { tail -30 $O/cifar_$amp.err; exit $rc; }
done
DET_GRAPH_HALF_DROPOUT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o cifar -- \
  python3 -u scripts/bench_cifar_trial.py --batch 32 --batches 1000 --chunk 500 --amp O2 --hip-graph --graph-batches 20 \
  --lr 1e-4 > $O/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $O/prof.log; exit 1; }
echo "prof done"
for v in bankmask none torch; do
  timeout -k 10 240 python -u scripts/dbg/chunk_vs_batch.py --variant $v --amp O2 --rounds 4 --out $O > $O/cvb_$v.log 2>&1 \
    || { echo "cvb $v rc=$?"; tail -30 $O/cvb_$v.log; exit 1; }
  echo "== cvb $v"; cut -c1-600 $O/cvb_$v.log
done
for cfg in "sep:--variant torch --separate-pools" "o0:--variant torch --amp O0" "nodrop:--variant none" \
           "bank:--variant bankmask" "native:--variant torch --native" "plain:--variant torch"; do
  name=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 240 python -u scripts/dbg/graph_nan_probe.py $a --graph-batches 20 --check-every 20 \
    --batches 3000 --out $O > $O/p_$name.json 2> $O/p_$name.err || { echo "$name failed rc=$?"; tail -30 $O/p_$name.err; exit 1; }
  echo "== $name $(python -c "
import json;d=json.load(open('$O/p_$name.json'))
print(d['batches_seen'], d['chunks_checked'], d['violation'], d['step_losses'], d['final_masters_finite'], d['wall_s'])")"
done
