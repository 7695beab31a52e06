#!/bin/bash
# Round-2 session 31: stem wgrad on MIOpen's C=4 kernel (native fwd + BN stats kept): numerics of both
# wgrad paths, ResNet-50 bench A/B (native stem on/off), steady-state kernel profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s31
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py > gpurun_out/s31/conv.log 2>&1 || { tail -40 gpurun_out/s31/conv.log; exit 1; }
tail -2 gpurun_out/s31/conv.log
timeout -k 10 400 python -u bench.py > gpurun_out/s31/bench.json 2> gpurun_out/s31/bench.err || { tail -20 gpurun_out/s31/bench.err; exit 1; }
cat gpurun_out/s31/bench.json
timeout -k 10 400 python -u bench.py --no-native-stem > gpurun_out/s31/bench_nostem.json 2> gpurun_out/s31/bench_nostem.err || { tail -20 gpurun_out/s31/bench_nostem.err; exit 1; }
cat gpurun_out/s31/bench_nostem.json
timeout -k 10 400 python -u bench.py > gpurun_out/s31/bench2.json 2> gpurun_out/s31/bench2.err || { tail -20 gpurun_out/s31/bench2.err; exit 1; }
cat gpurun_out/s31/bench2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s31/prof -o run -- python -u bench.py --steps 10 --warmup 5 > gpurun_out/s31/prof_bench.json 2> gpurun_out/s31/prof_bench.err || { tail -20 gpurun_out/s31/prof_bench.err; exit 1; }
python scripts/prof_summarize.py gpurun_out/s31/prof/run_results.db --step-kernel opt_kernel --skip-steps 3 --out gpurun_out/s31/steady.csv > gpurun_out/s31/steady.txt 2>&1 && rm -f gpurun_out/s31/prof/run_results.db
head -30 gpurun_out/s31/steady.txt
