#!/bin/bash
# Round-6 session 75: LayerNorm forward variants at the BERT shape (workgroup-per-row default vs the
# wave-per-row kernel, 1 / 2 rows per wave).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s75
mkdir -p $O
export TMPDIR=/tmp
for cfg in "DET_X=0" "DET_LN_FWD=narrow" "DET_LN_FWD=narrow DET_LN_ROWS=1" "DET_X=0" "DET_LN_FWD=narrow"; do
  env $cfg timeout -k 10 120 python -u scripts/bench_ln.py --iters 300 > $O/l.json 2> $O/l.err || { echo "ln rc=$?"; tail -20 $O/l.err; exit 1; }
  grep '^{' $O/l.json | tail -1 >> $O/ln.jsonl
  echo "$cfg: $(grep '^{' $O/l.json | tail -1 | grep -o '"fwd_us": [0-9.]*, "bwd_us": [0-9.]*')"
done
