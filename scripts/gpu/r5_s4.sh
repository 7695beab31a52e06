#!/bin/bash
# Round-5 session 4: (a) the round-4 NaN does not reproduce on this tree (s3: 6 replay runs clean).
# The one change on its path is the loss: round 4's train_batch ran torch's cross_entropy on
# out.float() and an argmax accuracy inside the graph, this tree one fused kernel.  Put the torch
# ops back (both, or one of them) on the round-4 model, asynchronous checks, 3 seeds.
# (b) native CIFAR CNN tests (split-K finish order fixed); (c) the CIFAR trial on the native kernels;
# (d) the ResNet-50 step baseline of this round: bench, steady profile, roofline vs det_stream, SQ counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s4
mkdir -p $O
export TMPDIR=/tmp
for cfg in "torch_s1:--loss torch --seed 1" "torch_s2:--loss torch --seed 2" "torch_s3:--loss torch --seed 3" \
           "torchce_s1:--loss torch_ce --seed 1" "torchacc_s1:--loss torch_acc --seed 1"; do
  name=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 240 python -u scripts/dbg/graph_nan_probe.py --variant torch --r4-model --check-every 100 $a --batches 2400 \
    --out $O > $O/$name.json 2> $O/$name.err || { echo "$name failed rc=$?"; tail -30 $O/$name.err; exit 1; }
  echo "== $name"; cut -c1-500 $O/$name.json
done
# a failed assertion (rc 1) lets the rest run; a fault / abort / timeout (any other rc) ends the call
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py -v --timeout 120 --timeout-method thread > $O/cnn_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/cnn_tests.log | head -20
[ $rc -le 1 ] || { tail -c 3000 $O/cnn_tests.log; exit $rc; }
if [ $rc -eq 0 ]; then
  for amp in O2 O0; do
    DET_GRAPH_HALF_DROPOUT=1 timeout -k 10 240 python -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 --amp $amp --hip-graph \
      --graph-batches 20 --lr 1e-4 > $O/cifar_$amp.json 2> $O/cifar_$amp.err
    rc=$?; echo "cifar $amp rc=$rc: $(cut -c1-400 $O/cifar_$amp.json)"
    [ $rc -le 1 ] || { tail -30 $O/cifar_$amp.err; exit $rc; }
  done
fi
for nt in 0 1 0 1; do  # BatchNorm apply passes with nontemporal activation reads (DET_BN_NT) A/B
  DET_BN_NT=$nt timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_nt$nt.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
  echo "bench DET_BN_NT=$nt $(cut -c1-160 $O/bench_nt$nt.json)"; cat $O/bench_nt$nt.json >> $O/bench_bn_nt_ab.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --steps 15 --warmup 5 \
  > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
python3 scripts/prof_summarize.py $(find $O/prof -name "bench_kernel_trace.csv" | head -1) --out $O/steady.csv > $O/steady.txt
head -45 $O/steady.txt
timeout -k 10 400 python -u scripts/step_roofline.py --iters 3 --out $O/step_roofline.csv > $O/step_roofline.txt 2>&1 || { tail -30 $O/step_roofline.txt; exit 1; }
sed -n '/per family/,$p' $O/step_roofline.txt | head -40
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace -d $O/pmc -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 3 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python3 scripts/pmc_summarize.py $(find $O/pmc -name "pmc_counter_collection.csv" | head -1) --top 30 --out $O/pmc_summary.csv > $O/pmc_summary.txt
head -35 $O/pmc_summary.txt
