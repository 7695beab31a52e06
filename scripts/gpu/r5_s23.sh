#!/bin/bash
# Round-5 session 23: tuned-GEMM + residual-link + graph-sink tests; BERT eager/graph with the shipped
# tuned GEMM file; BERT Linear shapes, vendor BLAS vs hand-written tiles; CIFAR steady profiles at the
# 512-block split-K default (O2, O0); ASHA O0 with normally-exiting containers under rocprofv3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s23
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_transformer_gpu.py -q --timeout 200 --timeout-method thread > $O/tf_tests.log 2>&1 || { tail -40 $O/tf_tests.log; exit 1; }
tail -1 $O/tf_tests.log
for g in "" "--hip-graph"; do
  timeout -k 10 300 python -u scripts/bench_bert.py --steps 60 --warmup 8 $g > $O/bert$g.json 2> $O/bert.err || { tail -12 $O/bert.err; exit 1; }
  echo "bert $g: $(cut -c1-120 $O/bert$g.json)"
done
timeout -k 10 200 python -u scripts/bench_linear_shapes.py > $O/linear_shapes.json 2> $O/linear.err || { tail -20 $O/linear.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/linear_shapes.json')); [print(k, v) for k, v in d['passes'].items()]"
for amp in O2 O0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/cprof_$amp -o cifar -- \
    python3 -u scripts/bench_cifar_trial.py --batch 32 --batches 2000 --chunk 500 --amp $amp --hip-graph --graph-batches 20 \
    --lr 1e-4 > $O/cifar_prof_$amp.json 2> $O/cifar_prof.err || { echo "cifar prof rc=$?"; tail -20 $O/cifar_prof.err; exit 1; }
  python3 scripts/prof_summarize.py $(find /tmp/cprof_$amp -name "*.db" | head -1) --step-kernel opt_kernel --skip-steps 200 --sequence \
    --out $O/cifar_steady_$amp.csv > $O/cifar_steady_$amp.txt
  head -3 $O/cifar_steady_$amp.txt
done
DET_FAST_EXIT=0 DET_BENCH_LOGDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/aprof -- python3 -u scripts/bench_asha.py \
  --slots 1 --amp O0 --graph-batches 20 --timeout 540 --no-zygote > $O/asha_prof.json 2> $O/asha_prof.err \
  || { echo "asha prof rc=$?"; tail -20 $O/asha_prof.err; exit 1; }
echo "asha prof: $(grep '^{' $O/asha_prof.json | tail -1 | cut -c1-300)"
find /tmp/aprof -name "*.db" > $O/asha_prof_dbs.txt; wc -l $O/asha_prof_dbs.txt
timeout -k 10 120 python3 scripts/prof_busy.py /tmp/aprof --out $O/asha_o0_rocprof_busy.json
