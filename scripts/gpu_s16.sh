#!/bin/bash
# Session: transformer kernel tests (H=4096 LN, tanh GELU, ALBERT), ALBERT-xxlarge bench + profile.
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
step pytest_tf 400 python -u -m pytest tests/test_transformer_gpu.py -x -v --timeout 200 --timeout-method thread
step albert1 500 python scripts/bench_albert.py --steps 12 --warmup 6
step bert1 300 python scripts/bench_bert.py --steps 30 --warmup 5
step prof_albert 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_albert1 -o albert --output-format csv -- python3 scripts/bench_albert.py --steps 6 --warmup 6
python scripts/prof_summarize.py $(ls gpurun_out/prof_albert1/*/albert_kernel_trace.csv gpurun_out/prof_albert1/albert_kernel_trace.csv 2>/dev/null | head -1) --skip-steps 2 --out gpurun_out/albert1_steady.csv > gpurun_out/albert1_steady.txt 2>&1 || true
grep -h metric gpurun_out/albert1.log gpurun_out/bert1.log | cut -c1-250
head -30 gpurun_out/albert1_steady.txt
echo "[session] done"
