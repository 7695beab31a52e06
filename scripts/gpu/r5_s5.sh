#!/bin/bash
# Round-5 session 5: (a) native CIFAR CNN tests (exact dropout test at scales 2/4, bf16 vs torch's
# own bf16 error, captured-step update vs fp32 same-mask recompute) and the CIFAR trial on them;
# (b) BatchNorm apply nontemporal-read A/B on the ResNet bench; (c) the O2 NaN with chunked (20)
# graphs on the round-4 model and loss path, 3 seeds x 3000 batches; (d) BERT hipGraph vs eager,
# 2000 steps, loss per 100.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s5
mkdir -p $O
export TMPDIR=/tmp
# a failed assertion (rc 1) lets the rest run; a fault / abort / timeout (any other rc) ends the call
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py -v --timeout 120 --timeout-method thread > $O/cnn_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/cnn_tests.log | head -20
[ $rc -le 1 ] || { tail -c 3000 $O/cnn_tests.log; exit $rc; }
if [ $rc -eq 0 ]; then
  for amp in O2 O0; do
    DET_GRAPH_HALF_DROPOUT=1 timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 \
      --amp $amp --hip-graph --graph-batches 20 --lr 1e-4 > $O/cifar_$amp.json 2> $O/cifar_$amp.err
    rc=$?; echo "cifar $amp rc=$rc: $(cut -c1-420 $O/cifar_$amp.json)"
    [ $rc -le 1 ] || { tail -30 $O/cifar_$amp.err; exit $rc; }
  done
else
  grep -E "^E  " $O/cnn_tests.log | grep -v "tensor(" | head -20
fi
for nt in 0 1 0 1; do
  DET_BN_NT=$nt timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_nt$nt.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
  echo "bench DET_BN_NT=$nt $(cut -c1-150 $O/bench_nt$nt.json)"; cat $O/bench_nt$nt.json >> $O/bench_bn_nt_ab.jsonl
done
for cfg in "g20_torch_s1:--loss torch --seed 1" "g20_torch_s2:--loss torch --seed 2" "g20_torch_s3:--loss torch --seed 3" \
           "g20_ref_s1:--seed 1"; do
  name=${cfg%%:*}; a=${cfg#*:}
  r4=""; [[ $name == *torch* ]] && r4="--r4-model"
  timeout -k 10 240 python -u scripts/dbg/graph_nan_probe.py --variant torch $r4 --graph-batches 20 --check-every 100 $a \
    --batches 3000 --out $O > $O/$name.json 2> $O/$name.err || { echo "$name failed rc=$?"; tail -30 $O/$name.err; exit 1; }
  echo "== $name $(cut -c1-700 $O/$name.json)"
done
for g in "" "--hip-graph"; do
  timeout -k 10 400 python -u scripts/bench_bert.py --steps 2000 --warmup 8 --loss-every 100 $g > $O/bert$g.json 2> $O/bert$g.err \
    || { tail -20 $O/bert$g.err; exit 1; }
  echo "bert $g $(cut -c1-130 $O/bert$g.json) $(grep -o '"graph_stats[^}]*}' $O/bert$g.json) $(grep -o '"losses.*' $O/bert$g.json | cut -c1-400)"
done
