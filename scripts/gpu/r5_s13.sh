#!/bin/bash
# Round-5 session 13: (a) CIFAR trial after exact-bf16 staging: speed + lean kernel trace + SQ
# counters (summaries only; raw traces deleted); (b) BERT hipGraph vs eager over 2000 steps (loss per
# 100, progress on stderr); (c) ResNet bench A/B of the BN-backward dgrad prefetch (DET_BNB_PF).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s13
mkdir -p $O
export TMPDIR=/tmp
for amp in O2 O0; do
  timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 \
    --amp $amp --hip-graph --graph-batches 20 --lr 1e-4 > $O/cifar_$amp.json 2> $O/cifar_$amp.err
  rc=$?; echo "cifar $amp rc=$rc: $(cut -c1-200 $O/cifar_$amp.json)"
  [ $rc -le 1 ] || { tail -30 $O/cifar_$amp.err; exit $rc; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/cprof -o cifar -- \
  python3 -u scripts/bench_cifar_trial.py --batch 32 --batches 1000 --chunk 500 --amp O2 --hip-graph --graph-batches 20 \
  --lr 1e-4 > $O/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $O/prof.log; exit 1; }
python3 scripts/prof_summarize.py $(find /tmp/cprof -name "*.db" | head -1) --step-kernel opt_kernel --skip-steps 200 \
  --out $O/cifar_steady.csv > $O/cifar_steady.txt 2>&1; head -45 $O/cifar_steady.txt
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
  --kernel-trace -d /tmp/cpmc -o pmc --output-format csv -- python3 -u scripts/bench_cifar_trial.py --batch 32 --batches 200 \
  --chunk 100 --amp O2 --hip-graph --graph-batches 20 --lr 1e-4 > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -20 $O/pmc.log; exit 1; }
python3 scripts/pmc_summarize.py $(find /tmp/cpmc -name "pmc_counter_collection.csv" | head -1) --top 30 --out $O/cifar_pmc.csv > $O/cifar_pmc.txt 2>&1
head -40 $O/cifar_pmc.txt
for g in "" "--hip-graph"; do
  timeout -k 10 420 python -u scripts/bench_bert.py --steps 2000 --warmup 8 --loss-every 100 $g > $O/bert$g.json 2> $O/bert$g.err \
    || { echo "bert $g rc=$?"; tail -20 $O/bert$g.err; exit 1; }
  echo "bert $g $(cut -c1-130 $O/bert$g.json) $(grep -o '"graph_stats[^}]*}' $O/bert$g.json) $(grep -o '"losses.*' $O/bert$g.json | cut -c1-300)"
done
for pf in 1 2 1 2; do
  DET_BN_NT=1 DET_BNB_PF=$pf timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_pf$pf.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
  echo "bench DET_BNB_PF=$pf $(cut -c1-150 $O/bench_pf$pf.json)"
done
