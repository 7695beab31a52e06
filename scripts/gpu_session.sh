#!/bin/bash
# One GPU-box session: build, GPU tests, bench, profile.  Every GPU step has its own timeout and
# the script stops at the first failure/fault (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[session] $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[session] $name rc=$rc" | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ]; then tail -30 "gpurun_out/$name.log"; exit $rc; fi
}
MODE=${1:-all}
step build 300 python -c "import __graft_entry__ as g; g.build()"
if [[ $MODE == all || $MODE == test ]]; then
  step pytest_gpu 600 python -m pytest tests -m gpu -x -q
fi
if [[ $MODE == all || $MODE == bench ]]; then
  step bench 400 python bench.py
fi
if [[ $MODE == all || $MODE == prof ]]; then
  export TMPDIR=/tmp
  step prof 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 5
fi
echo "[session] done"
