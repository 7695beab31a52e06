#!/bin/bash
# Round-6 session 1: the ADVICE r5 fixes on the GPU (transformer / cnn / embed / DP tests), smoke(),
# bench.py x2 and a steady-state ResNet-50 kernel profile as this round's starting point.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_transformer_gpu.py tests/test_cnn_gpu.py tests/test_embed_gpu.py tests/test_bert.py tests/test_graph_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $O/bench$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo "bench: $(cut -c1-150 $O/bench$i.json)"; cat $O/bench$i.json >> $O/bench.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --steps 15 --warmup 5 \
  > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
python3 scripts/prof_summarize.py $(find $O/prof -name "bench_kernel_trace.csv" | head -1) --out $O/steady.csv > $O/steady.txt
head -12 $O/steady.txt
