#!/bin/bash
# Round-5 session 15: native BERT embedding (graph-safe backward) tests, then BERT eager vs hipGraph
# over 2000 steps (the graph run faulted at ~700 replays in s13/s14 with torch's embedding backward);
# then the ResNet bench A/B of the BN-backward dgrad prefetch depth.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s15
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_embed_gpu.py tests/test_graph_cifar_o2_gpu.py::test_half_precision_library_convs_keep_train_batch_eager \
  -v --timeout 120 --timeout-method thread > $O/embed_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/embed_tests.log | head -20
[ $rc -eq 0 ] || { grep -E "^E  " $O/embed_tests.log | head -20; tail -c 2000 $O/embed_tests.log; exit 1; }
for g in "" "--hip-graph"; do
  timeout -k 10 300 python -u scripts/bench_bert.py --steps 2000 --warmup 8 --loss-every 100 $g > $O/bert$g.json 2> $O/bert$g.err
  rc=$?; echo "bert $g rc=$rc $(cut -c1-130 $O/bert$g.json) $(grep -o '"graph_stats[^}]*}' $O/bert$g.json) $(grep -o '"losses.*' $O/bert$g.json | cut -c1-300)"
  [ $rc -eq 0 ] || { tail -12 $O/bert$g.err; exit 1; }
done
# A/B: BN-backward dgrad prefetch (DET_BNB_PF) and the channel-fixed BN apply mapping (the nocf
# library is the same build with -DDET_BN_CF=0)
for cfg in "pf1_cf:1:" "pf2_cf:2:" "pf1_nocf:1:nocf" "pf1_cf:1:" "pf2_cf:2:" "pf1_nocf:1:nocf"; do
  name=${cfg%%:*}; rest=${cfg#*:}; pf=${rest%%:*}; v=${rest#*:}
  lib=""; [ "$v" = "nocf" ] && lib="DET_KERNELS_LIB=$PWD/determined_1_amd/ops/libdetkernels_nocf.so"
  env $lib DET_BN_NT=1 DET_BNB_PF=$pf timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_$name.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
  echo "bench $name $(cut -c1-150 $O/bench_$name.json)"; cat $O/bench_$name.json >> $O/bench_ab.jsonl
done
