#!/bin/bash
# Session: fused-QKV attention — numerics, BERT throughput, kernel profile.
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
step pytest_tf 400 python -m pytest tests/test_transformer_gpu.py -x -q
step bert1 300 python scripts/bench_bert.py --steps 30 --warmup 5
step bert2 300 python scripts/bench_bert.py --steps 30 --warmup 5
step prof_bert 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert3 -o bert --output-format csv -- python3 scripts/bench_bert.py --steps 12 --warmup 5
python scripts/prof_summarize.py $(ls gpurun_out/prof_bert3/*/bert_kernel_trace.csv gpurun_out/prof_bert3/bert_kernel_trace.csv 2>/dev/null | head -1) --skip-steps 4 --out gpurun_out/bert3_steady.csv > gpurun_out/bert3_steady.txt 2>&1 || true
grep -h metric gpurun_out/bert1.log gpurun_out/bert2.log | cut -c1-160
head -30 gpurun_out/bert3_steady.txt
echo "[session] done"
