#!/bin/bash
# Round-3 session 35: BN-backward epilogue loads hoisted before the K loop (gemm_nt BNB, occupancy 2);
# K == 64 variant A/B (DET_BNB_SINGLE_OCC), kernel tests, steady profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s35
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bn_bwd_fusion_gpu.py tests/test_conv_gpu.py tests/test_norm_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0 1 0; do
  DET_BNB_SINGLE_OCC=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 > $O/bench_single$v.json 2> $O/bench_single$v.err || { tail -30 $O/bench_single$v.err; exit 1; }
  echo "single=$v $(cut -c1-110 $O/bench_single$v.json)"
done
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/steady.csv > $O/steady.txt 2>&1 || { tail -5 $O/steady.txt; exit 1; }
head -12 $O/steady.txt
rm -rf $O/prof
