#!/bin/bash
# Round-5 session 14: (a) CIFAR CNN with the lane-group split-K finish: tests + speed + steady trace
# summary; (b) LAST: the BERT hipGraph run that faulted in s13 after ~700 replays (memory aperture
# violation), now with rocBLAS instead of hipBLASLt for torch's GEMMs, to see whether the fault follows
# hipBLASLt inside graphs.  Nothing runs after it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s14
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py -v --timeout 300 --timeout-method thread > $O/cnn_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/cnn_tests.log | head -30
[ $rc -le 1 ] || { tail -c 3000 $O/cnn_tests.log; exit $rc; }
[ $rc -eq 0 ] || { grep -E "^E  " $O/cnn_tests.log | grep -v "tensor(" | head -20; exit 1; }
for amp in O2 O0; do
  timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 \
    --amp $amp --hip-graph --graph-batches 20 --lr 1e-4 > $O/cifar_$amp.json 2> $O/cifar_$amp.err
  rc=$?; echo "cifar $amp rc=$rc: $(cut -c1-200 $O/cifar_$amp.json)"
  [ $rc -le 1 ] || { tail -30 $O/cifar_$amp.err; exit $rc; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/cprof -o cifar -- \
  python3 -u scripts/bench_cifar_trial.py --batch 32 --batches 1000 --chunk 500 --amp O2 --hip-graph --graph-batches 20 \
  --lr 1e-4 > $O/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $O/prof.log; exit 1; }
python3 scripts/prof_summarize.py $(find /tmp/cprof -name "*.db" | head -1) --step-kernel opt_kernel --skip-steps 200 \
  --out $O/cifar_steady.csv > $O/cifar_steady.txt 2>&1; head -30 $O/cifar_steady.txt
TORCH_BLAS_PREFER_HIPBLASLT=0 timeout -k 10 300 python -u scripts/bench_bert.py --steps 2000 --warmup 8 --loss-every 100 \
  --hip-graph > $O/bert_graph_rocblas.json 2> $O/bert_graph_rocblas.err
rc=$?; echo "bert graph rocblas rc=$rc $(cut -c1-130 $O/bert_graph_rocblas.json)"; tail -4 $O/bert_graph_rocblas.err
