#!/bin/bash
# Round-2 session 4: full GPU suite on the rebuilt tree; ResNet-50 bench A/B of the det_conv 1x1 GEMMs;
# steady-state kernel stats of the default path.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s4
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s4/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/s4/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s4/bench_native.json 2> gpurun_out/s4/bench_native.err || { tail -20 gpurun_out/s4/bench_native.err; exit 1; }
cat gpurun_out/s4/bench_native.json
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 --no-native-conv1x1 > gpurun_out/s4/bench_miopen.json 2> gpurun_out/s4/bench_miopen.err || { tail -20 gpurun_out/s4/bench_miopen.err; exit 1; }
cat gpurun_out/s4/bench_miopen.json
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d gpurun_out/s4/prof -o run -- python3 -u bench.py --steps 10 --warmup 5 > gpurun_out/s4/bench_prof.json 2> gpurun_out/s4/bench_prof.err || { tail -20 gpurun_out/s4/bench_prof.err; exit 1; }
cat gpurun_out/s4/bench_prof.json
exit $rc
