#!/bin/bash
# Round-6 session 60: where the LayerNorm backward's 20.5 us go at the BERT shape: kernel trace of
# scripts/bench_ln.py with dropout 0.1 and 0 (ln_bwd_kernel vs colsum_finalize vs ln_fwd).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s60
mkdir -p $O
export TMPDIR=/tmp
for p in 0.1 0; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_$p -o ln -- python3 -u scripts/bench_ln.py --iters 200 --p $p \
    > $O/ln_$p.log 2>&1 || { echo "prof p=$p rc=$?"; tail -20 $O/ln_$p.log; exit 1; }
  grep '^{' $O/ln_$p.log | grep -o '"fwd_us": [0-9.]*, "bwd_us": [0-9.]*'
done
