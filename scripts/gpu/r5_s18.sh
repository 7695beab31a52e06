#!/bin/bash
# Round-5 session 18: CNN tests after the conv2-split fix, CIFAR speed + steady sequence + SQ counters per wave.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s18
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py tests/test_graph_cifar_o2_gpu.py tests/test_graph_chunks.py -v --timeout 300 --timeout-method thread > $O/cnn_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/cnn_tests.log | head -30
[ $rc -le 1 ] || { tail -c 3000 $O/cnn_tests.log; exit $rc; }
[ $rc -eq 0 ] || { grep -E "^E  " $O/cnn_tests.log | head -20; exit 1; }
for amp in O2 O0; do
  timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 \
    --amp $amp --hip-graph --graph-batches 20 --lr 1e-4 > $O/cifar_$amp.json 2> $O/cifar_$amp.err
  rc=$?; echo "cifar $amp rc=$rc: $(cut -c1-200 $O/cifar_$amp.json)"
  [ $rc -le 1 ] || { tail -30 $O/cifar_$amp.err; exit $rc; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/cprof -o cifar -- \
  python3 -u scripts/bench_cifar_trial.py --batch 32 --batches 1000 --chunk 500 --amp O2 --hip-graph --graph-batches 20 \
  --lr 1e-4 > $O/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $O/prof.log; exit 1; }
python3 scripts/prof_summarize.py $(find /tmp/cprof -name "*.db" | head -1) --step-kernel opt_kernel --skip-steps 200 --sequence \
  --out $O/cifar_steady.csv > $O/cifar_steady.txt 2>&1; head -70 $O/cifar_steady.txt
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
  --kernel-trace -d /tmp/cpmc -o pmc --output-format csv -- python3 -u scripts/bench_cifar_trial.py --batch 32 --batches 200 \
  --chunk 100 --amp O2 --hip-graph --graph-batches 20 --lr 1e-4 > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -20 $O/pmc.log; exit 1; }
python3 scripts/pmc_per_wave.py $(find /tmp/cpmc -name "pmc_counter_collection.csv" | head -1) --top 25 --out $O/cifar_pmc_per_wave.txt
