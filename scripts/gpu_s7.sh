#!/bin/bash
# Session: ASHA trials/hr with per-trial harness timelines, then a rocprofv3 kernel profile of BERT.
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
  if [ $rc -ne 0 ]; then tail -40 "gpurun_out/$name.log"; exit $rc; fi
}
step build 400 python -c "import __graft_entry__ as g; g.build()"
step asha 700 env DET_BENCH_LOGDIR=gpurun_out python scripts/bench_asha.py --max-length-batches 300 --max-trials 16 --timeout 600
step prof_bert 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o bert --output-format csv -- python3 scripts/bench_bert.py --steps 12 --warmup 5
python scripts/prof_summarize.py $(ls gpurun_out/prof_bert/*/bert_kernel_trace.csv gpurun_out/prof_bert/bert_kernel_trace.csv 2>/dev/null | head -1) --skip-steps 4 --out gpurun_out/bert_steady.csv > gpurun_out/bert_steady.txt 2>&1 || true
grep metric gpurun_out/asha.log | cut -c1-800
head -40 gpurun_out/bert_steady.txt
echo "[session] done"
