#!/bin/bash
# Round-6 session 58: LayerNorm backward variants at the BERT shape (4608 x 768 bf16, dropout 0.1):
# the backward runs ~21 us per call in the BERT step against a ~6.4 us streaming bound.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s58
mkdir -p $O
export TMPDIR=/tmp
run() {
  env "$@" timeout -k 10 120 python -u scripts/bench_ln.py --iters 200 > $O/l.json 2> $O/l.err || { echo "ln $* rc=$?"; tail -20 $O/l.err; exit 1; }
  grep '^{' $O/l.json | tail -1 >> $O/ln.jsonl
  echo "$*: $(grep '^{' $O/l.json | tail -1 | cut -c1-330)"
}
run DET_X=0
run DET_LN_BWD_BLOCKS=256
run DET_LN_BWD_BLOCKS=1152
run DET_LN_BWD_BLOCKS=2304
run DET_LN_ROWS=1
run DET_LN_ROWS=1 DET_LN_BWD_BLOCKS=1152
run DET_LN_BWD=wide
run DET_LN_BWD=wide DET_LN_BWD_BLOCKS=1152
