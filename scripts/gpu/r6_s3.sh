#!/bin/bash
# Round-6 session 3: kernel-argument census of the captured bf16 MIOpen bwd-weight convs (which memory
# each kernel argument points into), DP / aggregation hipGraph capture on a world-1 RCCL group.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_graph_dp_gpu.py -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "FAILED|ERROR|Error" $O/tests.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/dbg/graph_nodes.py --dtype bf16 --args conv1_bwd_weight,conv2_bwd_weight,conv1_fwd > $O/args_bf16.jsonl 2> $O/args.err
arc=$?; echo "args rc=$arc"; grep bwd_weight $O/args_bf16.jsonl | cut -c1-1500; tail -3 $O/args.err
[ $arc -eq 0 ] || exit $arc
# igemm3 at two workgroups per CU (cfgs 16-20) on the ResNet-50 1x1 and 3x3 shapes and the BERT GEMMs
timeout -k 10 300 python -u scripts/bench_igemm_cfgs.py --cfgs 8,9,11,16,17,18,19,20 > $O/cfgs_1x1.jsonl 2> $O/cfgs.err || { tail -5 $O/cfgs.err; exit 1; }
for c in 0 16 19 20; do
  DET_IGEMM_CFG=$c timeout -k 10 300 python -u scripts/bench_conv3x3.py > $O/conv3x3_cfg$c.jsonl 2>> $O/cfgs.err || { tail -5 $O/cfgs.err; exit 1; }
  echo "3x3 cfg $c: $(tail -1 $O/conv3x3_cfg$c.jsonl | cut -c1-300)"
done
timeout -k 10 300 python -u scripts/bench_linear_shapes.py --igemm 8,9,16,19,20 --wgcfg 3,4,6,7 > $O/bert_shapes.json 2>> $O/cfgs.err || { tail -5 $O/cfgs.err; exit 1; }
echo done
