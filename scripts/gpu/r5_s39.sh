#!/bin/bash
# Round-5 session 39: cross-entropy gradient from the forward launch (fixed condition): CNN tests,
# CIFAR O2/O0, O2 steady profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s39
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py tests/test_graph_cifar_o2_gpu.py -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for amp in O2 O0 O2 O0; do
  timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 \
    --amp $amp --hip-graph --graph-batches 20 --lr 1e-4 > $O/cifar_$amp.json 2> $O/cifar.err || { tail -20 $O/cifar.err; exit 1; }
  echo "cifar $amp: $(cut -c1-100 $O/cifar_$amp.json)"; cat $O/cifar_$amp.json >> $O/cifar_runs.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cprof -o cifar -- \
  python3 -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 --amp O2 --hip-graph --graph-batches 20 \
  --lr 1e-4 > $O/cifar_prof.json 2> $O/cifar_prof.err || { echo "cifar prof rc=$?"; tail -20 $O/cifar_prof.err; exit 1; }
python3 scripts/prof_summarize.py $(find /tmp/cprof -name "*.db" | head -1) --step-kernel opt_kernel --skip-steps 200 --sequence \
  --out $O/cifar_steady_O2.csv > $O/cifar_steady_O2.txt
head -20 $O/cifar_steady_O2.txt
