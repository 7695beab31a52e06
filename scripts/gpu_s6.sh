#!/bin/bash
# Session: BERT-base throughput, then the ASHA trials/hr cluster benchmark on the GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[session] $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[session] $name rc=$rc" | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ]; then tail -40 "gpurun_out/$name.log"; exit $rc; fi
}
step build 400 python -c "import __graft_entry__ as g; g.build()"
step bert 400 env DET_STEP_TIMERS=1 python scripts/bench_bert.py --steps 20 --warmup 5
step asha 700 env DET_BENCH_LOGDIR=gpurun_out python scripts/bench_asha.py --max-length-batches 300 --max-trials 16 --timeout 600
for f in gpurun_out/bert.log gpurun_out/asha.log; do grep metric $f | cut -c1-400; done
echo "[session] done"
