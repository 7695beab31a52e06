#!/bin/bash
# Round-4 session 8: stem BN backward fused into the max-pool gather (partials) + the stem weight
# gradient (deferred apply); faster pool indexing; projection-shortcut BN apply deferred into bn3's
# (forward) and into the shortcut dgrad (backward); merged attention backward grid.  Tests, bench
# A/B (fusions on / off, bn-prologue), steady profile, per-call step roofline, attention microbench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s8
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_pool_gpu.py tests/test_conv_gpu.py tests/test_bn_bwd_fusion_gpu.py tests/test_norm_gpu.py tests/test_attention_gpu.py tests/test_transformer_gpu.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "on::" "off:DET_POOL_BN_BWD=0 DET_DEFER_AFFINE_APPLY=0:" "on::" "off:DET_POOL_BN_BWD=0 DET_DEFER_AFFINE_APPLY=0:" "pro::--bn-prologue"; do
  name=${cfg%%:*}; rest=${cfg#*:}; envs=${rest%%:*}; args=${rest#*:}
  env $envs timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 $args > $O/bench_$name.json 2> $O/bench_$name.err || { tail -30 $O/bench_$name.err; exit 1; }
  echo "$name $(python3 -c "import json;d=json.load(open('$O/bench_$name.json'));print(d['value'],d['ms_per_step'])")"
done
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/steady.csv > $O/steady.txt 2>&1 || { tail -5 $O/steady.txt; exit 1; }
head -3 $O/steady.txt
rm -rf $O/prof
timeout -k 10 300 python -u scripts/step_roofline.py --iters 3 --out $O/step_roofline.csv > $O/step_roofline.txt 2>&1 || { tail -30 $O/step_roofline.txt; exit 1; }
sed -n '/per family/,$p' $O/step_roofline.txt | head -40
timeout -k 10 300 python -u scripts/bench_attn.py --graph > $O/attn_graph.jsonl 2> $O/attn.err || { tail -20 $O/attn.err; exit 1; }
head -3 $O/attn_graph.jsonl | cut -c1-500
