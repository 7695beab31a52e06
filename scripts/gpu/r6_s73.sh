#!/bin/bash
# Round-6 session 73: the column-sum finalize (LayerNorm / bias gradients) with 64 (default), 32 or
# 16 columns per 1,024-thread block (DET_FIN_COLS): LN microbench, transformer tests, BERT graph A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s73
mkdir -p $O
export TMPDIR=/tmp
for c in 64 32 16; do
  DET_FIN_COLS=$c timeout -k 10 120 python -u scripts/bench_ln.py --iters 200 > $O/l.json 2> $O/l.err || { echo "ln rc=$?"; tail -20 $O/l.err; exit 1; }
  echo "ln cols=$c: $(grep '^{' $O/l.json | tail -1 | grep -o '"bwd_us": [0-9.]*')"
done
DET_FIN_COLS=16 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_transformer_gpu.py \
  > $O/test.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error" $O/test.log | head; tail -20 $O/test.log; exit 1; }
tail -1 $O/test.log
for rep in 1 2; do
  for c in 64 16 32; do
    DET_FIN_COLS=$c timeout -k 10 300 python -u scripts/bench_bert.py --steps 200 --warmup 10 --hip-graph \
      > $O/b.json 2> $O/b.err || { echo "bert cols=$c rc=$?"; tail -20 $O/b.err; exit 1; }
    line=$(grep '^{' $O/b.json | tail -1)
    echo "{\"fin_cols\": $c, \"bench\": $line}" >> $O/ab.jsonl
    echo "bert cols=$c: $(echo "$line" | grep -o '"value": [0-9.]*')"
  done
done
