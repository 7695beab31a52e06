#!/bin/bash
# Session: workgroup-per-row LayerNorm forward for every width, hardware bf16 packing in the
# transformer kernels, skipped no-op attention rescales — tests, BERT/ALBERT throughput, BERT profile.
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
step albert1 500 python scripts/bench_albert.py --steps 12 --warmup 6
grep -h metric gpurun_out/bert1.log gpurun_out/albert1.log | cut -c1-170
step prof_bert 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert8 -o bert --output-format csv -- python3 scripts/bench_bert.py --steps 12 --warmup 5
python3 scripts/kstats.py gpurun_out/prof_bert8/bert_kernel_stats.csv 40 17 > gpurun_out/bert8_top.txt 2>&1
grep -E "total|attn|ln_|gelu|col|opt_|mt_copy|Functor_add" gpurun_out/bert8_top.txt
rm -f gpurun_out/prof_bert8/bert_kernel_trace.csv
echo "[session] done"
