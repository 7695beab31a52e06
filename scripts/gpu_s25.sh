#!/bin/bash
# Session: full GPU test suite; ResNet-50 bs512 steady-state kernel profile after the stem pool /
# shortcut-link changes; BERT throughput regression check.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[session] $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[session] $name rc=$rc" | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ]; then tail -30 "gpurun_out/$name.log"; fi
  if [ $rc -gt 1 ]; then exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
step bert1 300 python scripts/bench_bert.py --steps 30 --warmup 5
grep -h metric gpurun_out/bert1.log | cut -c1-160
step prof_r50 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50b -o r50 --output-format csv -- python3 bench.py --steps 6 --warmup 10
python3 scripts/prof_summarize.py gpurun_out/prof_r50b/r50_kernel_trace.csv --skip-steps 3 --out gpurun_out/r50b_steady.csv > gpurun_out/r50b_steady.txt 2>&1
head -40 gpurun_out/r50b_steady.txt
rm -f gpurun_out/prof_r50b/r50_kernel_trace.csv
echo "[session] done"
