#!/bin/bash
# Session: TunableOp GEMM selection for the BERT shapes (tune once, then reuse the results file).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[session] $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[session] $name rc=$rc" | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ]; then tail -60 "gpurun_out/$name.log"; exit $rc; fi
}
step bert_base 300 python scripts/bench_bert.py --steps 30 --warmup 5
step bert_tune 600 env PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_bert.csv python scripts/bench_bert.py --steps 30 --warmup 5
step bert_tuned 300 env PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_bert.csv python scripts/bench_bert.py --steps 30 --warmup 5
step bert_base2 300 python scripts/bench_bert.py --steps 30 --warmup 5
grep -h metric gpurun_out/bert_base.log gpurun_out/bert_tune.log gpurun_out/bert_tuned.log gpurun_out/bert_base2.log | cut -c1-160
ls -la gpurun_out/tunableop_bert*.csv; head -20 gpurun_out/tunableop_bert*.csv
echo "[session] done"
