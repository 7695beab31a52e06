#!/bin/bash
# Session: BERT host-overhead study (phase timers incl. host issue time, cProfile).
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
step bert_timers 300 env DET_STEP_TIMERS=1 python scripts/bench_bert.py --steps 30 --warmup 5
step bert_cprof 400 python -m cProfile -o gpurun_out/bert.cprof scripts/bench_bert.py --steps 40 --warmup 5
python scripts/cprof_summary.py gpurun_out/bert.cprof 45 > gpurun_out/bert_cprof.txt 2>&1 || true
grep -E "phase timers|metric" gpurun_out/bert_timers.log | cut -c1-400
head -80 gpurun_out/bert_cprof.txt
echo "[session] done"
