#!/bin/bash
# Round-4 session 3: halo-patch 3x3 kernel (conv3p) numerics + pass timings, bench A/B (conv3p on /
# off), steady profile; then the ResNet DP equivalence tests (2 ranks sharing the GPU over gloo).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_conv3x3_gpu.py tests/test_conv_gpu.py tests/test_bn_bwd_fusion_gpu.py tests/test_norm_gpu.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u scripts/bench_conv3x3.py > $O/conv3x3.jsonl 2> $O/conv3x3.err || { tail -20 $O/conv3x3.err; exit 1; }
cut -c1-420 $O/conv3x3.jsonl
for v in 128 0 128 0; do
  DET_CONV3P_MAX_N=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_p3_$v.json 2> $O/bench_p3_$v.err || { tail -30 $O/bench_p3_$v.err; exit 1; }
  echo "conv3p_max_n=$v $(cut -c1-110 $O/bench_p3_$v.json)"
done
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/steady.csv > $O/steady.txt 2>&1 || { tail -5 $O/steady.txt; exit 1; }
head -3 $O/steady.txt
rm -rf $O/prof
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -p no:cacheprovider -m gpu tests/test_dp_resnet_gpu.py > $O/pytest_dp.log 2>&1 || { tail -60 $O/pytest_dp.log; exit 1; }
tail -3 $O/pytest_dp.log
