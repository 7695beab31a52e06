#!/bin/bash
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
step gemm 300 python scripts/bench_gemm.py
step bert_a 300 python scripts/bench_bert.py --steps 30 --warmup 5
step bert_b 300 python scripts/bench_bert.py --steps 30 --warmup 5
step bert_rocblas 300 env TORCH_BLAS_PREFER_HIPBLASLT=0 python scripts/bench_bert.py --steps 30 --warmup 5
cat gpurun_out/gemm.log | grep lib
grep -h metric gpurun_out/bert_a.log gpurun_out/bert_b.log gpurun_out/bert_rocblas.log | cut -c1-200
echo "[session] done"
