#!/bin/bash
# Round-5 session 43: global average pool + batched weight flips: their GPU tests and the conv/pool/BN/DP
# suites, bench A/B DET_DW_BATCH 1/0 (alternating), and a steady-state kernel profile of the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s43
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pool_gpu.py tests/test_conv3x3_gpu.py tests/test_conv_gpu.py tests/test_bn_bwd_fusion_gpu.py tests/test_dp_resnet_gpu.py tests/test_examples_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
[ $rc -le 1 ] || exit $rc
for b in 1 0 1 0; do
  DET_DW_BATCH=$b timeout -k 10 300 python -u bench.py > $O/bench_dw$b.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo "bench DET_DW_BATCH=$b $(cut -c1-150 $O/bench_dw$b.json)"; cat $O/bench_dw$b.json >> $O/bench_dw_ab.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --steps 15 --warmup 5 \
  > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
python3 scripts/prof_summarize.py $(find $O/prof -name "bench_kernel_trace.csv" | head -1) --out $O/steady.csv > $O/steady.txt
head -45 $O/steady.txt
