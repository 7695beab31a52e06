#!/bin/bash
# Round-3 session 33: native projection shortcuts (1x1 stride 1/2 with BN stats, stride-2 gradient
# kept on its grid): kernel tests, microbench vs MIOpen, bench A/B, steady profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s33
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_bn_bwd_fusion_gpu.py tests/test_conv_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u scripts/bench_shortcut.py > $O/shortcut.jsonl 2> $O/shortcut.err || { tail -20 $O/shortcut.err; exit 1; }
cat $O/shortcut.jsonl
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 > $O/bench_on.json 2> $O/bench_on.err || { tail -30 $O/bench_on.err; exit 1; }
cut -c1-120 $O/bench_on.json
DET_NATIVE_SHORTCUT=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 > $O/bench_off.json 2> $O/bench_off.err || { tail -30 $O/bench_off.err; exit 1; }
cut -c1-120 $O/bench_off.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 > $O/bench_on2.json 2> $O/bench_on2.err || { tail -30 $O/bench_on2.err; exit 1; }
cut -c1-120 $O/bench_on2.json
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/steady.csv > $O/steady.txt 2>&1 || { tail -5 $O/steady.txt; exit 1; }
head -3 $O/steady.txt
rm -rf $O/prof
