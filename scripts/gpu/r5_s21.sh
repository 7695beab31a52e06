#!/bin/bash
# Round-5 session 21: residual-gradient link tests; BERT eager/graph with the link; hipBLASLt solution
# tuning (PyTorch TunableOp) of the BERT GEMM shapes, then eager/graph again from the tuned file.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s21
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_transformer_gpu.py tests/test_graph_gpu.py tests/test_graph_chunks.py tests/test_graph_dropout_gpu.py \
  tests/test_embed_gpu.py -q --timeout 200 --timeout-method thread > $O/tf_tests.log 2>&1 || { tail -40 $O/tf_tests.log; exit 1; }
tail -1 $O/tf_tests.log
DET_GRAPH_SINK=0 timeout -k 10 300 python -u scripts/bench_bert.py --steps 60 --warmup 8 --hip-graph > $O/bert_link_nosink.json 2> $O/bert.err || { tail -12 $O/bert.err; exit 1; }
echo "bert link graph, no sink: $(cut -c1-120 $O/bert_link_nosink.json)"
for g in "" "--hip-graph"; do
  timeout -k 10 300 python -u scripts/bench_bert.py --steps 60 --warmup 8 $g > $O/bert_link$g.json 2> $O/bert.err || { tail -12 $O/bert.err; exit 1; }
  echo "bert link $g: $(cut -c1-120 $O/bert_link$g.json)"
done
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tunableop_bert.csv \
  timeout -k 10 900 python -u scripts/bench_bert.py --steps 20 --warmup 3 > $O/bert_tuning.json 2> $O/bert_tuning.err \
  || { echo "tuning rc=$?"; tail -30 $O/bert_tuning.err; exit 1; }
echo "bert while tuning: $(cut -c1-120 $O/bert_tuning.json)"
ls -la $O/ | grep -i tunable
F=$(ls $O/tunableop_bert*.csv | head -1)
wc -l $F
for g in "" "--hip-graph"; do
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$PWD/$F \
    timeout -k 10 300 python -u scripts/bench_bert.py --steps 60 --warmup 8 $g > $O/bert_tuned$g.json 2> $O/bert.err || { tail -12 $O/bert.err; exit 1; }
  echo "bert tuned $g: $(cut -c1-120 $O/bert_tuned$g.json)"
done
DET_BENCH_LOGDIR=$O timeout -k 10 600 python -u scripts/bench_asha.py --slots 1 --amp O0 --graph-batches 20 --timeout 540 \
  > $O/asha_O0.json 2> $O/asha_O0.err || { echo "asha O0 rc=$?"; tail -20 $O/asha_O0.err; exit 1; }
echo "asha O0: $(grep '^{' $O/asha_O0.json | tail -1 | cut -c1-300)"
# one rocpd database per process (no -o: the default name carries the pid)
DET_BENCH_LOGDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/aprof -- python3 -u scripts/bench_asha.py \
  --slots 1 --amp O0 --graph-batches 20 --timeout 540 --no-zygote > $O/asha_prof.json 2> $O/asha_prof.err \
  || { echo "asha prof rc=$?"; tail -20 $O/asha_prof.err; exit 1; }
echo "asha prof: $(grep '^{' $O/asha_prof.json | tail -1 | cut -c1-300)"
find /tmp/aprof -name "*.db" | head -30 > $O/asha_prof_dbs.txt
timeout -k 10 120 python3 scripts/prof_busy.py /tmp/aprof --out $O/asha_o0_rocprof_busy.json
