#!/bin/bash
# A/B session: numerics of the BN kernels, then bench variants (AMP level, MIOpen find mode).
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
step bench_o1 400 python bench.py
step bench_o2 400 env DET_BENCH_AMP=O2 python bench.py
step bench_o1_find 500 env DET_BENCH_CUDNN_BENCHMARK=1 python bench.py
grep -h metric gpurun_out/bench_o*.log | cut -c1-200
echo "[session] done"
