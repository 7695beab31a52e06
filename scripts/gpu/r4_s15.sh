#!/bin/bash
# Round-4 session 15: statistics-epilogue order A/B on one box (DET_STATS_FIRST), hipGraph for
# Adam (device-side lr / bias corrections) -- graph tests and the BERT bench -- and the roofline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s15
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_conv_gpu.py tests/test_igemm_gpu.py tests/test_conv3x3_gpu.py tests/test_bn_bwd_fusion_gpu.py tests/test_graph_gpu.py tests/test_kernels_gpu.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 0 1 0 1; do
  DET_STATS_FIRST=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_sf$v.json 2> $O/bench_sf$v.err || { tail -30 $O/bench_sf$v.err; exit 1; }
  echo "bench stats_first=$v $(python3 -c "import json;d=json.load(open('$O/bench_sf$v.json'));print(d['value'],d['ms_per_step'])")"
  cat $O/bench_sf$v.json >> $O/bench_ab.jsonl
done
for g in "" "--hip-graph"; do
  timeout -k 10 400 python -u scripts/bench_bert.py --steps 30 --warmup 8 $g > $O/bert$g.json 2> $O/bert$g.err || { tail -20 $O/bert$g.err; exit 1; }
  echo "bert $g $(cut -c1-110 $O/bert$g.json) $(grep -o '"graph_stats[^}]*}' $O/bert$g.json)"
done
timeout -k 10 300 python -u scripts/step_roofline.py --iters 3 --out $O/step_roofline.csv > $O/step_roofline.txt 2>&1 || { tail -30 $O/step_roofline.txt; exit 1; }
sed -n '/per family/,$p' $O/step_roofline.txt | head -34
