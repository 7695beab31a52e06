#!/bin/bash
# Round-3 session 6: BN-backward fusion into the 1x1 dgrad epilogue: numerics, ResNet grads A/B, bench, profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3s6
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_bwd_fusion_gpu.py tests/test_conv_gpu.py tests/test_norm_gpu.py tests/test_conv3x3_gpu.py > gpurun_out/r3s6/pytest.log 2>&1 || { tail -40 gpurun_out/r3s6/pytest.log; exit 1; }
tail -2 gpurun_out/r3s6/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 > gpurun_out/r3s6/bench.json 2> gpurun_out/r3s6/bench.err || { tail -30 gpurun_out/r3s6/bench.err; exit 1; }
cat gpurun_out/r3s6/bench.json
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3s6/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > gpurun_out/r3s6/bench_prof.json 2> gpurun_out/r3s6/bench_prof.err || { tail -20 gpurun_out/r3s6/bench_prof.err; exit 1; }
f=$(find gpurun_out/r3s6/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out gpurun_out/r3s6/steady.csv > gpurun_out/r3s6/steady.txt 2>&1 || { tail -5 gpurun_out/r3s6/steady.txt; exit 1; }
head -30 gpurun_out/r3s6/steady.txt
rm -rf gpurun_out/r3s6/prof
