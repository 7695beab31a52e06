#!/bin/bash
# Round-6 session 80: kernel trace of the final default bench step (1,024 images/GPU, side stream, wgrad8).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s80
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 12 --warmup 8 \
  > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
grep '^{' $O/prof.log | cut -c1-200
