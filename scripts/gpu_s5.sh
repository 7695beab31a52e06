#!/bin/bash
# Session: bench (bs512 default, bitmask BN), bs256 reference, steady-state profile, BERT bench.
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
step pytest_norm 300 python -m pytest tests/test_norm_gpu.py -x -q
step bench_default 500 python bench.py
export TMPDIR=/tmp
step prof_default 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o bench --output-format csv -- python3 bench.py --steps 12 --warmup 6
step bert 400 python scripts/bench_bert.py --steps 20 --warmup 5
for f in gpurun_out/bench_default.log gpurun_out/bert.log; do grep metric $f | cut -c1-200; done
echo "[session] done"
