#!/bin/bash
# Session: ALBERT shared-weight GEMM accumulation; TunableOp A/B on BERT + ALBERT.
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
step pytest_albert 300 python -u -m pytest tests/test_transformer_gpu.py -x -v --timeout 200 --timeout-method thread -k "albert or bert_layer or gelu"
step albert2 500 python scripts/bench_albert.py --steps 12 --warmup 6
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=0
export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_bert%d.csv
step bert_tuned 600 python scripts/bench_bert.py --steps 30 --warmup 10
export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_albert%d.csv
step albert_tuned 900 python scripts/bench_albert.py --steps 12 --warmup 6
grep -h metric gpurun_out/albert2.log gpurun_out/bert_tuned.log gpurun_out/albert_tuned.log | cut -c1-200
ls -la gpurun_out/*.csv
echo "[session] done"
