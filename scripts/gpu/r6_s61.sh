#!/bin/bash
# Round-6 session 61: LayerNorm backward with 16-B lanes (ln_bwd_v8_kernel, default) vs the 4-column
# lanes (DET_LN_BWD_V8=0): transformer GPU tests, the LN microbench, BERT graph bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s61
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_transformer_gpu.py \
  > $O/test.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error" $O/test.log | head; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 1 0; do
  DET_LN_BWD_V8=$v timeout -k 10 120 python -u scripts/bench_ln.py --iters 200 > $O/l.json 2> $O/l.err || { echo "ln rc=$?"; tail -20 $O/l.err; exit 1; }
  echo "ln v8=$v: $(grep '^{' $O/l.json | tail -1 | grep -o '"bwd_us": [0-9.]*')"
  grep '^{' $O/l.json | tail -1 >> $O/ln.jsonl
done
for rep in 1 2; do
  for v in 0 1; do
    DET_LN_BWD_V8=$v timeout -k 10 300 python -u scripts/bench_bert.py --steps 200 --warmup 10 --hip-graph \
      > $O/b.json 2> $O/b.err || { echo "bert v8=$v rc=$?"; tail -20 $O/b.err; exit 1; }
    line=$(grep '^{' $O/b.json | tail -1)
    echo "{\"ln_bwd_v8\": $v, \"bench\": $line}" >> $O/ab.jsonl
    echo "bert v8=$v: $(echo "$line" | grep -o '"value": [0-9.]*')"
  done
done
