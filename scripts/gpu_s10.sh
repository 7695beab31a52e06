#!/bin/bash
# Session: BERT host overhead — autograd threading A/B, steady-state cProfile.
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
step bert_mt 300 env DET_STEP_TIMERS=1 python scripts/bench_bert.py --steps 30 --warmup 5
step bert_st 300 env DET_STEP_TIMERS=1 python scripts/bench_bert.py --steps 30 --warmup 5 --autograd-threads 0
step bert_plain 300 python scripts/bench_bert.py --steps 30 --warmup 5
step bert_cprof 300 python scripts/bench_bert.py --steps 30 --warmup 5 --autograd-threads 0 --cprof gpurun_out/bert_st.cprof
python scripts/cprof_summary.py gpurun_out/bert_st.cprof 50 > gpurun_out/bert_st_cprof.txt 2>&1 || true
grep -E "phase timers|metric" gpurun_out/bert_mt.log gpurun_out/bert_st.log gpurun_out/bert_plain.log | cut -c1-330
head -75 gpurun_out/bert_st_cprof.txt
echo "[session] done"
