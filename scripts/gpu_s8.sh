#!/bin/bash
# Session: fused transformer kernels — numerics, BERT native vs HF throughput, kernel profile.
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
step build 300 python -m determined_1_amd.ops.build --force
step pytest_tf 400 python -m pytest tests/test_transformer_gpu.py -x -q
step bert_native 300 python scripts/bench_bert.py --steps 20 --warmup 5 --impl native
step bert_hf 300 python scripts/bench_bert.py --steps 20 --warmup 5 --impl hf
step prof_bert 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert2 -o bert --output-format csv -- python3 scripts/bench_bert.py --steps 12 --warmup 5 --impl native
python scripts/prof_summarize.py $(ls gpurun_out/prof_bert2/*/bert_kernel_trace.csv gpurun_out/prof_bert2/bert_kernel_trace.csv 2>/dev/null | head -1) --skip-steps 4 --out gpurun_out/bert2_steady.csv > gpurun_out/bert2_steady.txt 2>&1 || true
grep metric gpurun_out/bert_native.log gpurun_out/bert_hf.log | cut -c1-600
head -30 gpurun_out/bert2_steady.txt
echo "[session] done"
