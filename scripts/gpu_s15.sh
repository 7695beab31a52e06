#!/bin/bash
# Session: ResNet-50 bench (heartbeat), BERT throughput + kernel profile with MFMA attention.
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
step bench_r50 600 python bench.py --steps 30 --warmup 10
step bert1 300 python scripts/bench_bert.py --steps 30 --warmup 5
step prof_bert 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert5 -o bert --output-format csv -- python3 scripts/bench_bert.py --steps 12 --warmup 5
python scripts/prof_summarize.py $(ls gpurun_out/prof_bert5/*/bert_kernel_trace.csv gpurun_out/prof_bert5/bert_kernel_trace.csv 2>/dev/null | head -1) --skip-steps 4 --out gpurun_out/bert5_steady.csv > gpurun_out/bert5_steady.txt 2>&1 || true
grep -h metric gpurun_out/bert1.log gpurun_out/bench_r50.log | cut -c1-200
head -30 gpurun_out/bert5_steady.txt
echo "[session] done"
