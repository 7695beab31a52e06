#!/bin/bash
# Fused-BN session: numerics tests, A/B bench vs stock MIOpen BN, kernel profile.
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
step pytest_norm 400 python -m pytest tests/test_norm_gpu.py -x -q
step bench_fused 400 python bench.py
step bench_stock 400 python bench.py --no-fused-bn
export TMPDIR=/tmp
step prof_fused 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fused -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 5
step pytest_gpu 600 python -m pytest tests -m gpu -x -q
echo "[session] done"
