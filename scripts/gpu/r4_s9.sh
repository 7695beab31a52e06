#!/bin/bash
# Round-4 session 9: step roofline (read-stream reference on det_bn_stats_train); BERT-base SQuAD re-bench
# (hipBLASLt vs hand-written dense layers) on the current attention kernels (+ aggregation 2)
# with a steady rocprof profile; the ResNet DP equivalence tests (2 ranks sharing the GPU, gloo).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s9
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_pool_gpu.py tests/test_conv_gpu.py -k "stem or pool" > $O/pytest_stem.log 2>&1 || { tail -40 $O/pytest_stem.log; exit 1; }
tail -2 $O/pytest_stem.log
timeout -k 10 300 python -u scripts/step_roofline.py --iters 3 --out $O/step_roofline.csv > $O/step_roofline.txt 2>&1 || { tail -30 $O/step_roofline.txt; exit 1; }
sed -n '/per family/,$p' $O/step_roofline.txt | head -40
timeout -k 10 400 python -u scripts/bench_bert.py --steps 30 --warmup 8 > $O/bert.json 2> $O/bert.err || { tail -20 $O/bert.err; exit 1; }
echo "bert $(cut -c1-200 $O/bert.json)"
timeout -k 10 400 python -u scripts/bench_bert.py --steps 30 --warmup 8 --agg 2 > $O/bert_agg2.json 2> $O/bert_agg2.err || { tail -20 $O/bert_agg2.err; exit 1; }
echo "bert agg2 $(cut -c1-200 $O/bert_agg2.json)"
DET_NATIVE_LINEAR=1 timeout -k 10 400 python -u scripts/bench_bert.py --steps 30 --warmup 8 > $O/bert_nlin.json 2> $O/bert_nlin.err || { tail -20 $O/bert_nlin.err; exit 1; }
echo "bert native-linear $(cut -c1-200 $O/bert_nlin.json)"
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u scripts/bench_bert.py --steps 10 --warmup 8 > $O/bert_prof.json 2> $O/bert_prof.err || { tail -20 $O/bert_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/bert_steady.csv > $O/bert_steady.txt 2>&1 || { tail -5 $O/bert_steady.txt; exit 1; }
head -16 $O/bert_steady.txt
rm -rf $O/prof
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread -p no:cacheprovider -m gpu tests/test_dp_resnet_gpu.py > $O/pytest_dp.log 2>&1 || { tail -60 $O/pytest_dp.log; exit 1; }
grep "dp-vs-single\|passed\|failed" $O/pytest_dp.log | tail -6
timeout -k 10 300 python -u scripts/probe_small_launches.py --steps 3 --warmup 3 > $O/small_launches.txt 2>&1 || { tail -20 $O/small_launches.txt; exit 1; }
grep -A3 "copy_\|add\|fill" $O/small_launches.txt | head -30
