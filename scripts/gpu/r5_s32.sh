#!/bin/bash
# Round-5 session 32: BERT 2000 steps eager vs hipGraph with the GradSink capture path and the
# residual link (losses tracked every 100 steps); ALBERT-xxlarge bench; BERT eager host profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s32
mkdir -p $O
export TMPDIR=/tmp
for g in "" "--hip-graph"; do
  timeout -k 10 400 python -u scripts/bench_bert.py --steps 2000 --warmup 8 --loss-every 100 $g > $O/bert2000$g.json 2> $O/bert2000$g.err
  rc=$?; echo "bert2000 $g rc=$rc $(grep -o '"value": [0-9.]*' $O/bert2000$g.json) $(grep -o '"losses.*' $O/bert2000$g.json | cut -c1-200)"
  [ $rc -eq 0 ] || { tail -12 $O/bert2000$g.err; exit 1; }
done
timeout -k 10 400 python -u scripts/bench_albert.py > $O/albert.json 2> $O/albert.err || { tail -12 $O/albert.err; exit 1; }
echo "albert: $(cut -c1-200 $O/albert.json)"
timeout -k 10 300 python -u scripts/bench_bert.py --steps 40 --warmup 8 --cprof $O/bert_eager.cprof > $O/bert_cprof.json 2> $O/bert.err || { tail -12 $O/bert.err; exit 1; }
python3 scripts/cprof_summary.py $O/bert_eager.cprof 40 > $O/bert_eager_cprof.txt 2>&1
echo "bert eager under cProfile: $(grep -o '"value": [0-9.]*' $O/bert_cprof.json)"
