#!/bin/bash
# Round-5 session 25: LayerNorm kernel variants at the BERT-base shape (wave-per-row forward, two rows
# per wave iteration, backward grid), CNN finish with per-job lane groups + cached loss seed, tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s25
mkdir -p $O
export TMPDIR=/tmp
for cfg in "wide:1:512" "wide:2:512" "narrow:1:512" "narrow:2:512" "narrow:2:1024" "narrow:2:2048" "wide:2:1024"; do
  f=${cfg%%:*}; rest=${cfg#*:}; rr=${rest%%:*}; bl=${rest#*:}
  DET_LN_FWD=$f DET_LN_ROWS=$rr DET_LN_BWD_BLOCKS=$bl timeout -k 10 120 python -u scripts/bench_ln.py >> $O/ln_ab.jsonl 2> $O/ln.err || { tail -20 $O/ln.err; exit 1; }
  tail -1 $O/ln_ab.jsonl
done
timeout -k 10 600 python -u -m pytest tests/test_transformer_gpu.py tests/test_cnn_gpu.py tests/test_graph_gpu.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for amp in O2 O0; do
  timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 \
    --amp $amp --hip-graph --graph-batches 20 --lr 1e-4 > $O/cifar_$amp.json 2> $O/cifar.err || { tail -20 $O/cifar.err; exit 1; }
  echo "cifar $amp: $(cut -c1-100 $O/cifar_$amp.json)"
done
