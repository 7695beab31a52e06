#!/bin/bash
# O2 sweep: batch size, MIOpen find mode, and a kernel profile of the default config.
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
step bench_o2 400 python bench.py
step bench_o2_find 500 env DET_BENCH_CUDNN_BENCHMARK=1 python bench.py
step bench_o2_bs384 400 env DET_BENCH_BS=384 python bench.py
step bench_o2_bs512 500 env DET_BENCH_BS=512 python bench.py
export TMPDIR=/tmp
step prof_o2 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_o2 -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 5
grep -h metric gpurun_out/bench_o2*.log | cut -c1-160
echo "[session] done"
