#!/bin/bash
# Round-4 session 1: baseline on this box -- pool/link tests, DET_MAXPOOL_LINK A/B (interleaved), steady profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_pool_gpu.py > $O/pytest_pool.log 2>&1 || { tail -40 $O/pytest_pool.log; exit 1; }
tail -1 $O/pytest_pool.log
for v in 1 0 1 0 1 0; do
  DET_MAXPOOL_LINK=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_link$v.json 2> $O/bench_link$v.err || { tail -30 $O/bench_link$v.err; exit 1; }
  echo "link=$v $(cut -c1-120 $O/bench_link$v.json)"
done
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(ls $O/prof/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/steady.csv > $O/steady.txt 2>&1 || { tail -5 $O/steady.txt; exit 1; }
head -3 $O/steady.txt
rm -rf $O/prof
