#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
DET_SYNC_DEBUG=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -m pytest tests/test_norm_gpu.py -x -v -s -k "case3 or case0" > gpurun_out/dbg_norm.log 2>&1
echo "rc=$?"
tail -30 gpurun_out/dbg_norm.log
