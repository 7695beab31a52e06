#!/bin/bash
# Round-3 session 25/26: deferred BN-backward apply (ABN, coefficients hoisted per K tile; s26: expansion convs only): A/B bench
# (DET_DEFER_BN_APPLY=0/1) + steady profile of the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s26
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_bwd_fusion_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 0 1 0 1; do
  DET_DEFER_BN_APPLY=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 > $O/bench_defer$v.json 2> $O/bench_defer$v.err || { tail -30 $O/bench_defer$v.err; exit 1; }
  echo "defer=$v $(cut -c1-120 $O/bench_defer$v.json)"
  cat $O/bench_defer$v.json >> $O/bench_ab.jsonl
done
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/steady.csv > $O/steady.txt 2>&1 || { tail -5 $O/steady.txt; exit 1; }
head -16 $O/steady.txt
rm -rf $O/prof
