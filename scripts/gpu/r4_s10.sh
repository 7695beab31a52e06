#!/bin/bash
# Round-4 session 10: (+ stem patch forward and pool-forward A/Bs, roofline, PMC pass, BERT hipGraph)
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
DET_STEM_PATCH_FWD=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_stemgemm.json 2> $O/bench_stemgemm.err || { tail -30 $O/bench_stemgemm.err; exit 1; }
echo "bench stem-gemm $(python3 -c "import json;d=json.load(open('$O/bench_stemgemm.json'));print(d['value'],d['ms_per_step'])")"
DET_POOL_FWD_ROWS=1 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_poolrows.json 2> $O/bench_poolrows.err || { tail -30 $O/bench_poolrows.err; exit 1; }
echo "bench pool-fwd-rows $(python3 -c "import json;d=json.load(open('$O/bench_poolrows.json'));print(d['value'],d['ms_per_step'])")"
timeout -k 10 300 python -u scripts/step_roofline.py --iters 3 --out $O/step_roofline.csv > $O/step_roofline.txt 2>&1 || { tail -30 $O/step_roofline.txt; exit 1; }
grep -i "stem\|maxpool" $O/step_roofline.txt | head -12
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 8 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/steady.csv > $O/steady.txt 2>&1 || { tail -5 $O/steady.txt; exit 1; }
head -3 $O/steady.txt
rm -rf $O/prof
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o run -- python3 -u bench.py --steps 2 --warmup 2 > $O/pmc_bench.json 2> $O/pmc_bench.err || { tail -20 $O/pmc_bench.err; exit 1; }
f=$(find $O/pmc -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_summarize.py "$f" --top 40 --out $O/pmc_summary.csv > $O/pmc_summary.txt 2>&1 || { tail -5 $O/pmc_summary.txt; exit 1; }
head -25 $O/pmc_summary.txt
rm -rf $O/pmc
timeout -k 10 400 python -u scripts/bench_bert.py --steps 30 --warmup 8 --hip-graph > $O/bert_graph.json 2> $O/bert_graph.err || { tail -20 $O/bert_graph.err; exit 1; }
echo "bert hip_graph $(cut -c1-400 $O/bert_graph.json)"
for cfg in "gb20:" "o0:--amp O0"; do
  name=${cfg%%:*}; args=${cfg#*:}
  mkdir -p $O/asha_$name && DET_BENCH_LOGDIR=$O/asha_$name timeout -k 10 360 python -u scripts/bench_asha.py --slots 1 $args > $O/asha_$name.json 2> $O/asha_$name.err || { tail -30 $O/asha_$name.err; exit 1; }
  echo "asha $name $(cut -c1-300 $O/asha_$name.json)"
done
