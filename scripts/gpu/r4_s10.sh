#!/bin/bash
# Round-4 session 10: stem BN + ReLU applied inside the max-pool forward, max-pool backward with all
# window operands loaded up front: tests, bench x2, steady profile; then ASHA trials/hr on one GPU
# slot (the r3 default hip_graph_batches 20, and the reference precision O0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s10
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_pool_gpu.py tests/test_bn_bwd_fusion_gpu.py tests/test_conv_gpu.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_$i.json 2> $O/bench_$i.err || { tail -30 $O/bench_$i.err; exit 1; }
  echo "bench $i $(python3 -c "import json;d=json.load(open('$O/bench_$i.json'));print(d['value'],d['ms_per_step'])")"
done
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/steady.csv > $O/steady.txt 2>&1 || { tail -5 $O/steady.txt; exit 1; }
head -3 $O/steady.txt
rm -rf $O/prof
for cfg in "gb20:" "o0:--amp O0"; do
  name=${cfg%%:*}; args=${cfg#*:}
  mkdir -p $O/asha_$name && DET_BENCH_LOGDIR=$O/asha_$name timeout -k 10 360 python -u scripts/bench_asha.py --slots 1 $args > $O/asha_$name.json 2> $O/asha_$name.err || { tail -30 $O/asha_$name.err; exit 1; }
  echo "asha $name $(cut -c1-300 $O/asha_$name.json)"
done
