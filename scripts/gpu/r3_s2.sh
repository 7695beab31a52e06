#!/bin/bash
# Round-3 session 2: 3x3 conv path GPU tests + ResNet-50 bench A/B (native 3x3 vs MIOpen).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3s2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py tests/test_igemm_gpu.py > gpurun_out/r3s2/pytest.log 2>&1 || { tail -40 gpurun_out/r3s2/pytest.log; exit 1; }
tail -3 gpurun_out/r3s2/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 > gpurun_out/r3s2/bench_native3x3.json 2> gpurun_out/r3s2/bench_native3x3.err || { tail -30 gpurun_out/r3s2/bench_native3x3.err; exit 1; }
cat gpurun_out/r3s2/bench_native3x3.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 --no-native-conv3x3 > gpurun_out/r3s2/bench_miopen3x3.json 2> gpurun_out/r3s2/bench_miopen3x3.err || { tail -30 gpurun_out/r3s2/bench_miopen3x3.err; exit 1; }
cat gpurun_out/r3s2/bench_miopen3x3.json
