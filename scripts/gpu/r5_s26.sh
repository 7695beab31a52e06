#!/bin/bash
# Round-5 session 26: colsum finalize with 8x the blocks and 8 independent chains -- LN microbench,
# transformer tests, BERT eager / graph.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s26
mkdir -p $O
export TMPDIR=/tmp
for cfg in "wide:1:512" "narrow:1:512" "wide:1:256" "narrow:2:256"; do
  f=${cfg%%:*}; rest=${cfg#*:}; rr=${rest%%:*}; bl=${rest#*:}
  DET_LN_FWD=$f DET_LN_ROWS=$rr DET_LN_BWD_BLOCKS=$bl timeout -k 10 120 python -u scripts/bench_ln.py >> $O/ln_ab.jsonl 2> $O/ln.err || { tail -20 $O/ln.err; exit 1; }
  tail -1 $O/ln_ab.jsonl
done
timeout -k 10 600 python -u -m pytest tests/test_transformer_gpu.py tests/test_albert.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for g in "" "--hip-graph" "" "--hip-graph"; do
  timeout -k 10 300 python -u scripts/bench_bert.py --steps 60 --warmup 8 $g > $O/bert.json 2> $O/bert.err || { tail -12 $O/bert.err; exit 1; }
  echo "{\"graph\": \"$g\", \"result\": $(grep '^{' $O/bert.json | tail -1)}" >> $O/bert_ab.jsonl
  echo "bert $g: $(grep -o '"value": [0-9.]*' $O/bert.json)"
done
