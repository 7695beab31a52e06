#!/bin/bash
# Round-4 session 2: native stride-2 3x3 input gradient (parity-class implicit GEMMs): numerics,
# the linked-gradient guard / hook tests, 3x3 pass timings vs MIOpen, bench + steady profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_conv3x3_gpu.py tests/test_norm_gpu.py tests/test_bn_bwd_fusion_gpu.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u scripts/bench_conv3x3.py > $O/conv3x3.jsonl 2> $O/conv3x3.err || { tail -20 $O/conv3x3.err; exit 1; }
cut -c1-400 $O/conv3x3.jsonl
for v in 1 0 1; do
  DET_DGRAD_S2_NATIVE=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_s2_$v.json 2> $O/bench_s2_$v.err || { tail -30 $O/bench_s2_$v.err; exit 1; }
  echo "s2native=$v $(cut -c1-110 $O/bench_s2_$v.json)"
done
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/steady.csv > $O/steady.txt 2>&1 || { tail -5 $O/steady.txt; exit 1; }
head -3 $O/steady.txt
rm -rf $O/prof
