#!/bin/bash
# Round-5 session 33: cached-plan hipBLASLt path for the transformer Linears (det_blaslt.hip): tests,
# same-box BERT eager/graph A/B against torch.mm, eager host profile, ALBERT.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s33
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_transformer_gpu.py tests/test_albert.py tests/test_bert.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in "1:" "0:" "1:--hip-graph" "0:--hip-graph" "1:" "0:"; do
  bl=${cfg%%:*}; g=${cfg#*:}
  DET_BLASLT=$bl timeout -k 10 300 python -u scripts/bench_bert.py --steps 60 --warmup 8 $g > $O/bert.json 2> $O/bert.err || { tail -12 $O/bert.err; exit 1; }
  echo "{\"DET_BLASLT\": $bl, \"graph\": \"$g\", \"result\": $(grep '^{' $O/bert.json | tail -1)}" >> $O/bert_ab.jsonl
  echo "blaslt=$bl $g: $(grep -o '"value": [0-9.]*' $O/bert.json)"
done
timeout -k 10 300 python -u scripts/bench_bert.py --steps 40 --warmup 8 --cprof $O/bert_eager.cprof > $O/bert_cprof.json 2> $O/bert.err || { tail -12 $O/bert.err; exit 1; }
python3 scripts/cprof_summary.py $O/bert_eager.cprof 30 > $O/bert_eager_cprof.txt 2>&1
timeout -k 10 400 python -u scripts/bench_albert.py > $O/albert.json 2> $O/albert.err || { tail -12 $O/albert.err; exit 1; }
echo "albert: $(grep -o '"value": [0-9.]*' $O/albert.json)"
