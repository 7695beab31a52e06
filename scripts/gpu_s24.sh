#!/bin/bash
# Session: shortcut-link numerics debug; kernel tests (wide LayerNorm, pool, norm, 2-rank GPU-sharing
# DP smoke); ResNet-50 bench (HIP max-pool + shortcut links + cheaper BN apply VALU); ALBERT bench
# (wide LayerNorm); MIOpen asm NHWC wrw/bwd solvers off A/B.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...   (test failures continue; faults / timeouts / signals stop the session)
  local name=$1 t=$2; shift 2
  echo "[session] $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[session] $name rc=$rc" | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ]; then tail -30 "gpurun_out/$name.log"; fi
  if [ $rc -gt 1 ]; then exit $rc; fi
}
step dbg_link 200 python scripts/dbg_link.py
step pytest_k 600 python -u -m pytest tests/test_transformer_gpu.py tests/test_pool_gpu.py tests/test_norm_gpu.py tests/test_smoke_gpu.py -v --timeout 300 --timeout-method thread
step bench_r50 600 python bench.py --steps 30 --warmup 10
step albert1 500 python scripts/bench_albert.py --steps 12 --warmup 6
grep -h metric gpurun_out/bench_r50.log gpurun_out/albert1.log | cut -c1-180
grep -E "PASSED|FAILED" gpurun_out/pytest_k.log | grep -c PASSED
grep FAILED gpurun_out/pytest_k.log | head
cat gpurun_out/dbg_link.log | grep -v amdgpu
export MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0
step bench_r50_noasm 600 python bench.py --steps 30 --warmup 10
grep -h metric gpurun_out/bench_r50_noasm.log | cut -c1-150
echo "[session] done"
