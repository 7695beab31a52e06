#!/bin/bash
# Round-3 session 32: does the GPU test tier change the following bench? bench -> tier -> bench,
# then a steady profile of the post-tier state.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s32
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 > $O/bench_fresh.json 2> $O/bench_fresh.err || { tail -30 $O/bench_fresh.err; exit 1; }
cut -c1-120 $O/bench_fresh.json
ls -la /tmp/det-miopen-*/ 2>/dev/null | head; du -sh /tmp/det-miopen-* 2>/dev/null
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ls -la /tmp/det-miopen-*/ 2>/dev/null | head; du -sh /tmp/det-miopen-* 2>/dev/null
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 > $O/bench_after.json 2> $O/bench_after.err || { tail -30 $O/bench_after.err; exit 1; }
cut -c1-120 $O/bench_after.json
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/steady.csv > $O/steady.txt 2>&1 || { tail -5 $O/steady.txt; exit 1; }
head -3 $O/steady.txt
rm -rf $O/prof
