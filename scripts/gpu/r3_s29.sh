#!/bin/bash
# Round-3 session 29: deferred bn3 forward apply staged by the next block's conv1 (AFWD): numerics, ResNet tests, bench x2, profile.
# numerics (conv + ResNet fused-vs-stock), bench x2, steady profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s29
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_bwd_fusion_gpu.py tests/test_conv_gpu.py tests/test_norm_gpu.py tests/test_examples_gpu.py tests/test_smoke_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 > $O/bench$i.json 2> $O/bench$i.err || { tail -30 $O/bench$i.err; exit 1; }
  cut -c1-140 $O/bench$i.json
done
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/steady.csv > $O/steady.txt 2>&1 || { tail -5 $O/steady.txt; exit 1; }
head -12 $O/steady.txt
rm -rf $O/prof
