#!/bin/bash
# Round-6 session 4: where the DP hipGraph worker crashes (faulthandler), the BERT GEMM shapes on
# the igemm tiles, the 3x3 sweep at two workgroups per CU.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_linear_shapes.py --igemm 8,9,16,19,20 --wgcfg 3,4,6,7 > $O/bert_shapes.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
for c in 0 16 19 20; do
  DET_IGEMM_CFG=$c timeout -k 10 300 python -u scripts/bench_conv3x3.py > $O/conv3x3_cfg$c.jsonl 2>> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  echo "3x3 cfg $c: $(tail -1 $O/conv3x3_cfg$c.jsonl | cut -c1-300)"
done
# last: the crashing DP graph worker, once, with a Python traceback on the fault
env WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29577 DET_FORCE_DISTRIBUTED=1 \
  DET_HIP_GRAPH=1 GDP_HALF_STEPS=16 PYTHONFAULTHANDLER=1 \
  timeout -k 10 200 python -u tests/dist_scripts/gpu_dp_worker.py $O/dpg O2 1 0 fp32_accum > $O/dp_graph.log 2>&1
echo "dp graph worker rc=$?"; tail -40 $O/dp_graph.log
