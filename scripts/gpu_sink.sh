#!/bin/bash
# GradSink session: GPU tests, A/B bench (sink on/off), bs512, kernel profile.
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
step build 300 python -m determined_1_amd.ops.build --force
step pytest_gpu 600 python -m pytest tests -m gpu -x -q
step bench_sink 500 python bench.py
step bench_nosink 500 env DET_GRAD_SINK=0 python bench.py
step bench_bs512 600 env DET_BENCH_BS=512 python bench.py
export TMPDIR=/tmp
step prof_sink 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sink -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 5
for f in gpurun_out/bench_*.log; do echo $f; grep metric $f | cut -c1-150; done
echo "[session] done"
