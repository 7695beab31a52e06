#!/bin/bash
# Round-3 session 4: hybrid 3x3 (native fwd + s1 dgrad, MIOpen wgrad) tests, bench, steady profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3s4
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py > gpurun_out/r3s4/pytest.log 2>&1 || { tail -40 gpurun_out/r3s4/pytest.log; exit 1; }
tail -2 gpurun_out/r3s4/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 > gpurun_out/r3s4/bench.json 2> gpurun_out/r3s4/bench.err || { tail -30 gpurun_out/r3s4/bench.err; exit 1; }
cat gpurun_out/r3s4/bench.json
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3s4/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > gpurun_out/r3s4/bench_prof.json 2> gpurun_out/r3s4/bench_prof.err || { tail -20 gpurun_out/r3s4/bench_prof.err; exit 1; }
f=$(find gpurun_out/r3s4/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out gpurun_out/r3s4/steady.csv > gpurun_out/r3s4/steady.txt 2>&1 || { tail -5 gpurun_out/r3s4/steady.txt; exit 1; }
head -40 gpurun_out/r3s4/steady.txt
rm -rf gpurun_out/r3s4/prof
