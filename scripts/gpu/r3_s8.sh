#!/bin/bash
# Round-3 session 8: BN-backward fusion (shortcut-link gating fix), generic MFMA attention tests,
# multi-batch hipGraph chunks, ResNet bench + steady profile, attention microbench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s8
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_bwd_fusion_gpu.py > $O/pytest_bn.log 2>&1 || { tail -40 $O/pytest_bn.log; exit 1; }
tail -2 $O/pytest_bn.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graph_chunks.py tests/test_graph_gpu.py > $O/pytest_attn.log 2>&1 || { tail -40 $O/pytest_attn.log; exit 1; }
tail -2 $O/pytest_attn.log
timeout -k 10 300 python -u scripts/bench_attn.py > $O/bench_attn.jsonl 2> $O/bench_attn.err || { tail -20 $O/bench_attn.err; exit 1; }
cat $O/bench_attn.jsonl
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/steady.csv > $O/steady.txt 2>&1 || { tail -5 $O/steady.txt; exit 1; }
head -30 $O/steady.txt
rm -rf $O/prof
