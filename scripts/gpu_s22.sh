#!/bin/bash
# Session: HIP stem max-pool + identity-shortcut gradient links — numerics and ResNet-50 bench;
# then an A/B with MIOpen's asm implicit-GEMM NHWC wrw/bwd solvers disabled (they zero-fill).
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
step pytest_norm 400 python -u -m pytest tests/test_norm_gpu.py tests/test_pool_gpu.py tests/test_smoke_gpu.py -x -v --timeout 300 --timeout-method thread
step bench_r50 600 python bench.py --steps 30 --warmup 10
grep -h metric gpurun_out/bench_r50.log | cut -c1-150
export MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0
step bench_r50_noasm 600 python bench.py --steps 30 --warmup 10
grep -h metric gpurun_out/bench_r50_noasm.log | cut -c1-150
echo "[session] done"
