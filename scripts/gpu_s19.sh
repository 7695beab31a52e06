#!/bin/bash
# Session: tiled MFMA attention backward — numerics, BERT/ALBERT throughput, BERT profile.
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
step pytest_attn 300 python -u -m pytest tests/test_transformer_gpu.py -x -v --timeout 200 --timeout-method thread -k "attention or bert_layer or albert"
step bert1 300 python scripts/bench_bert.py --steps 30 --warmup 5
step albert1 500 python scripts/bench_albert.py --steps 12 --warmup 6
step prof_bert 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert7 -o bert --output-format csv -- python3 scripts/bench_bert.py --steps 12 --warmup 5
python scripts/kstats.py gpurun_out/prof_bert7/bert_kernel_stats.csv 30 17 > gpurun_out/bert7_top.txt 2>&1 || true
grep -h metric gpurun_out/bert1.log gpurun_out/albert1.log | cut -c1-200
grep attn gpurun_out/bert7_top.txt
echo "[session] done"
