#!/bin/bash
# Round-5 session 28: LayerNorm backward variants at the BERT shape -- wave-per-row (default) vs
# workgroup-per-row with 16-B vectors (DET_LN_BWD=wide), grid size, dropout on/off; per-kernel times.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s28
mkdir -p $O
export TMPDIR=/tmp
for cfg in "narrow:512:0.1" "wide:512:0.1" "wide:1024:0.1" "wide:2048:0.1" "narrow:512:0" "wide:1024:0"; do
  bw=${cfg%%:*}; rest=${cfg#*:}; bl=${rest%%:*}; p=${rest#*:}
  DET_LN_BWD=$bw DET_LN_BWD_BLOCKS=$bl timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lp_$bw$bl$p -o ln -- \
    python3 -u scripts/bench_ln.py --iters 200 --p $p > $O/ln.json 2> $O/ln.err || { tail -20 $O/ln.err; exit 1; }
  f=$(find /tmp/lp_$bw$bl$p -name "*kernel_stats.csv" | head -1)
  echo "$cfg $(python3 -c "
import csv, json
d = json.load(open('$O/ln.json'))
rows = {r['Name'].split('(')[0].split('::')[-1][:24]: round(float(r['AverageNs']) / 1e3, 2) for r in csv.DictReader(open('$f'))}
print(d['fwd_us'], d['bwd_us'], {k: v for k, v in rows.items() if 'ln_' in k or 'colsum' in k})
")" | tee -a $O/ln_bwd_ab.txt
done
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -q -k "layernorm or layer_norm or bert_layer" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
DET_LN_BWD=wide timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -q -k "layernorm or layer_norm or bert_layer" --timeout 200 --timeout-method thread > $O/tests_wide.log 2>&1 || { tail -40 $O/tests_wide.log; exit 1; }
tail -1 $O/tests_wide.log
