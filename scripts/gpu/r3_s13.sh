#!/bin/bash
# Round-3 session 13: det_igemm_wgrad (ring + transposed reads) numerics per cfg, wgrad microbench vs
# gemm_tn / MIOpen, det_igemm cfg sweep on the 1x1 forward / input-gradient shapes, ResNet bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s13
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py -k "ring_wgrad" > $O/pytest_wgrad.log 2>&1 || { tail -40 $O/pytest_wgrad.log; exit 1; }
tail -2 $O/pytest_wgrad.log
timeout -k 10 400 python -u scripts/bench_wgrad.py > $O/wgrad.jsonl 2> $O/wgrad.err || { tail -20 $O/wgrad.err; exit 1; }
grep best $O/wgrad.jsonl; tail -1 $O/wgrad.jsonl
timeout -k 10 400 python -u scripts/bench_igemm_cfgs.py > $O/igemm_cfgs_1x1.jsonl 2> $O/igemm_cfgs_1x1.err || { tail -20 $O/igemm_cfgs_1x1.err; exit 1; }
tail -1 $O/igemm_cfgs_1x1.jsonl
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
