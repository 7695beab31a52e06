#!/bin/bash
# Round-5 session 24: small Linear passes on the hand-written tiles (DET_NATIVE_LINEAR=auto) -- tests,
# then a same-box BERT A/B (native auto vs library, tuned file on/off, eager and graph); an eager
# host profile; the post-GradSink graph-mode steady kernel profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s24
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_transformer_gpu.py tests/test_attention_gpu.py -q --timeout 200 --timeout-method thread > $O/tf_tests.log 2>&1 || { tail -40 $O/tf_tests.log; exit 1; }
tail -1 $O/tf_tests.log
for cfg in "auto:1:" "0:1:" "auto:0:" "auto:1:--hip-graph" "0:1:--hip-graph" "auto:0:--hip-graph" "auto:1:" "0:1:"; do
  nl=${cfg%%:*}; rest=${cfg#*:}; tg=${rest%%:*}; g=${rest#*:}
  DET_NATIVE_LINEAR=$nl DET_TUNED_GEMMS=$tg timeout -k 10 300 python -u scripts/bench_bert.py --steps 60 --warmup 8 $g \
    > $O/bert.json 2> $O/bert.err || { tail -12 $O/bert.err; exit 1; }
  echo "{\"native_linear\": \"$nl\", \"tuned\": $tg, \"graph\": \"$g\", \"result\": $(grep '^{' $O/bert.json | tail -1)}" >> $O/bert_ab.jsonl
  echo "native=$nl tuned=$tg $g: $(grep -o '"value": [0-9.]*' $O/bert.json)"
done
timeout -k 10 300 python -u scripts/bench_bert.py --steps 40 --warmup 8 --cprof $O/bert_eager.cprof > $O/bert_cprof.json 2> $O/bert.err || { tail -12 $O/bert.err; exit 1; }
python3 scripts/cprof_summary.py $O/bert_eager.cprof 45 > $O/bert_eager_cprof.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/bprof -o bert -- python3 -u scripts/bench_bert.py --steps 80 --warmup 8 \
  --hip-graph > $O/bert_graph_prof.json 2> $O/bert_graph_prof.err || { echo "bert prof rc=$?"; tail -20 $O/bert_graph_prof.err; exit 1; }
python3 scripts/prof_summarize.py $(find /tmp/bprof -name "*.db" | head -1) --step-kernel opt_kernel --skip-steps 30 \
  --out $O/bert_graph_steady.csv > $O/bert_graph_steady.txt
head -30 $O/bert_graph_steady.txt | cut -c1-150
