#!/bin/bash
# Round-5 session 44: the whole GPU suite + smoke() with the round's last kernels (head pool, batched
# flips, 4-pixel input normalize), bench.py x2 and a steady-state kernel profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s44
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.log 2>&1
rc=$?; tail -2 $O/gpu_suite.log; grep -E "FAILED|ERROR" $O/gpu_suite.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $O/bench$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo "bench: $(cut -c1-150 $O/bench$i.json)"; cat $O/bench$i.json >> $O/bench.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --steps 15 --warmup 5 \
  > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
python3 scripts/prof_summarize.py $(find $O/prof -name "bench_kernel_trace.csv" | head -1) --out $O/steady.csv > $O/steady.txt
head -3 $O/steady.txt; grep -E "u8_normalize|gap_|dgrad_weight" $O/steady.txt
