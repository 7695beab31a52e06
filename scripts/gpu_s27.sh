#!/bin/bash
# Session: direct gradient landing (dW GEMMs write into the arena) — numerics test, BERT/ALBERT
# throughput (BERT twice: box-to-box variance check), 2-rank GPU-sharing BERT DP smoke.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[session] $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[session] $name rc=$rc" | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ]; then tail -30 "gpurun_out/$name.log"; fi
  if [ $rc -gt 1 ]; then exit $rc; fi
}
step pytest_tf 400 python -u -m pytest tests/test_transformer_gpu.py -v --timeout 200 --timeout-method thread
grep -E "passed|failed" gpurun_out/pytest_tf.log | tail -1
step bert1 300 python scripts/bench_bert.py --steps 30 --warmup 5
step bert2 300 python scripts/bench_bert.py --steps 60 --warmup 10
step albert1 500 python scripts/bench_albert.py --steps 12 --warmup 6
grep -h metric gpurun_out/bert1.log gpurun_out/bert2.log gpurun_out/albert1.log | cut -c1-170
DET_DIST_SHARE_GPU=1 DET_DIST_BACKEND=gloo step bert_dp2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 scripts/bench_bert.py --steps 3 --warmup 2 --agg 2
grep -h metric gpurun_out/bert_dp2.log | cut -c1-170
echo "[session] done"
