#!/bin/bash
# Round-5 session 7: (a) native CIFAR CNN after specialising the gather-GEMM per job kind (BK 64,
# vector LDS stores, unrolled split-K finish): tests, trial speed O2/O0 and a kernel trace; (b) which
# library op mis-replays in a 20-step graph (per-op bf16 graphs vs eager; whole steps with and
# without cudnn.deterministic; fp32 control).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py -v --timeout 120 --timeout-method thread > $O/cnn_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/cnn_tests.log | head -20
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
timeout -k 10 300 python -u scripts/dbg/miopen_graph_repro.py --k 20 --replays 5 > $O/ops_bf16.log 2>&1 || { echo "ops rc=$?"; tail -20 $O/ops_bf16.log; exit 1; }
echo "== ops bf16"; grep -v Warning $O/ops_bf16.log | cut -c1-260
timeout -k 10 300 python -u scripts/dbg/miopen_graph_repro.py --k 20 --replays 5 --deterministic > $O/ops_bf16_det.log 2>&1 || { echo "ops det rc=$?"; tail -20 $O/ops_bf16_det.log; exit 1; }
echo "== ops bf16 deterministic"; tail -1 $O/ops_bf16_det.log
for a in "" "--deterministic" "--dtype fp32"; do
  timeout -k 10 300 python -u scripts/dbg/miopen_graph_repro.py --step --k 20 --replays 8 $a > $O/step.log 2>&1 || { echo "step rc=$?"; tail -20 $O/step.log; exit 1; }
  echo "== step $a"; grep '"mode"' $O/step.log | cut -c1-220
done
