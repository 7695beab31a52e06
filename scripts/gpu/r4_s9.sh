#!/bin/bash
# Round-4 session 9: ResNet-50 per-call step roofline (read/write stream bounds); BERT-base SQuAD
# re-bench on the round-3 attention kernels (+ aggregation 2) with a steady rocprof profile; the
# attention microbench timed as hipGraph replays (GPU time, not host launch rate), merged backward
# grid vs two launches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s9
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_attention_gpu.py tests/test_transformer_gpu.py > $O/pytest_attn.log 2>&1 || { tail -40 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
timeout -k 10 300 python -u scripts/step_roofline.py --iters 3 --out $O/step_roofline.csv > $O/step_roofline.txt 2>&1 || { tail -30 $O/step_roofline.txt; exit 1; }
sed -n '/per family/,$p' $O/step_roofline.txt
timeout -k 10 300 python -u scripts/bench_attn.py --graph > $O/attn_graph.jsonl 2> $O/attn.err || { tail -20 $O/attn.err; exit 1; }
head -3 $O/attn_graph.jsonl | cut -c1-400
timeout -k 10 400 python -u scripts/bench_bert.py --steps 30 --warmup 8 > $O/bert.json 2> $O/bert.err || { tail -20 $O/bert.err; exit 1; }
echo "bert $(cut -c1-200 $O/bert.json)"
timeout -k 10 400 python -u scripts/bench_bert.py --steps 30 --warmup 8 --agg 2 > $O/bert_agg2.json 2> $O/bert_agg2.err || { tail -20 $O/bert_agg2.err; exit 1; }
echo "bert agg2 $(cut -c1-200 $O/bert_agg2.json)"
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u scripts/bench_bert.py --steps 10 --warmup 8 > $O/bert_prof.json 2> $O/bert_prof.err || { tail -20 $O/bert_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/bert_steady.csv > $O/bert_steady.txt 2>&1 || { tail -5 $O/bert_steady.txt; exit 1; }
head -16 $O/bert_steady.txt
rm -rf $O/prof
