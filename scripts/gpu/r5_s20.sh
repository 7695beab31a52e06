#!/bin/bash
# Round-5 session 20: CIFAR split-K sizing at O0 (and 256 at O2) with the new 512 default; ASHA O0
# trials/hr; ASHA O0 again with cold-exec containers under rocprofv3 (kernel-trace GPU-busy); BERT
# hipGraph steady-state kernel profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s20
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py -q --timeout 300 --timeout-method thread > $O/cnn_tests.log 2>&1 || { tail -30 $O/cnn_tests.log; exit 1; }
tail -1 $O/cnn_tests.log
for cfg in O0:512 O0:256 O0:1024 O2:256 O2:512; do
  amp=${cfg%%:*}; b=${cfg#*:}
  DET_CNN_BLOCKS=$b timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 \
    --amp $amp --hip-graph --graph-batches 20 --lr 1e-4 > $O/cifar_${amp}_b$b.json 2> $O/cifar.err || { tail -20 $O/cifar.err; exit 1; }
  echo "$amp blocks $b: $(cut -c1-100 $O/cifar_${amp}_b$b.json)"
done
DET_BENCH_LOGDIR=$O timeout -k 10 600 python -u scripts/bench_asha.py --slots 1 --amp O0 --graph-batches 20 --timeout 540 \
  > $O/asha_O0.json 2> $O/asha_O0.err || { echo "asha O0 rc=$?"; tail -20 $O/asha_O0.err; exit 1; }
echo "asha O0: $(grep '^{' $O/asha_O0.json | tail -1 | cut -c1-300)"
DET_BENCH_LOGDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/aprof -o asha -- python3 -u scripts/bench_asha.py \
  --slots 1 --amp O0 --graph-batches 20 --timeout 540 --no-zygote > $O/asha_prof.json 2> $O/asha_prof.err \
  || { echo "asha prof rc=$?"; tail -20 $O/asha_prof.err; exit 1; }
echo "asha prof: $(grep '^{' $O/asha_prof.json | tail -1 | cut -c1-300)"
timeout -k 10 120 python3 scripts/prof_busy.py /tmp/aprof --out $O/asha_o0_rocprof_busy.json
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/bprof -o bert -- python3 -u scripts/bench_bert.py --steps 80 --warmup 8 \
  --hip-graph > $O/bert_graph_prof.json 2> $O/bert_graph_prof.err || { echo "bert prof rc=$?"; tail -20 $O/bert_graph_prof.err; exit 1; }
echo "bert graph prof: $(cut -c1-150 $O/bert_graph_prof.json)"
python3 scripts/prof_summarize.py $(find /tmp/bprof -name "*.db" | head -1) --step-kernel opt_kernel --skip-steps 30 \
  --out $O/bert_graph_steady.csv > $O/bert_graph_steady.txt
head -40 $O/bert_graph_steady.txt | cut -c1-160
