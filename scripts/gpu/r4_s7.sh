#!/bin/bash
# Round-4 session 7: register prefetch depth of the plain 1x1 GEMMs (det_conv_nt PF 1..3): exact
# numerics at every depth, per-shape 1x1 timings (GEMM-only and fused, vs MIOpen), bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_conv_gpu.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u scripts/bench_conv1x1.py > $O/conv1x1.jsonl 2> $O/conv1x1.err || { tail -20 $O/conv1x1.err; exit 1; }
tail -1 $O/conv1x1.jsonl
for v in 1 2 3 1 2 3; do
  DET_NT_PF=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_pf$v.json 2> $O/bench_pf$v.err || { tail -30 $O/bench_pf$v.err; exit 1; }
  echo "pf=$v $(cut -c1-110 $O/bench_pf$v.json)"
done
timeout -k 10 300 python -u scripts/step_roofline.py --iters 3 --out $O/step_roofline.csv > $O/step_roofline.txt 2>&1 || { tail -30 $O/step_roofline.txt; exit 1; }
sed -n '/per family/,$p' $O/step_roofline.txt
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/steady.csv > $O/steady.txt 2>&1 || { tail -5 $O/steady.txt; exit 1; }
head -3 $O/steady.txt
rm -rf $O/prof
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -p no:cacheprovider -m gpu tests/test_dp_resnet_gpu.py > $O/pytest_dp.log 2>&1 || { tail -60 $O/pytest_dp.log; exit 1; }
tail -3 $O/pytest_dp.log
