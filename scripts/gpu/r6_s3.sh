#!/bin/bash
# Round-6 session 3: kernel-argument census of the captured bf16 MIOpen bwd-weight convs (which memory
# each kernel argument points into), DP / aggregation hipGraph capture on a world-1 RCCL group.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/dbg/graph_nodes.py --dtype bf16 --args conv1_bwd_weight,conv2_bwd_weight,conv1_fwd > $O/args_bf16.jsonl 2> $O/args.err; echo "args rc=$?"
grep bwd_weight $O/args_bf16.jsonl | cut -c1-1500; tail -3 $O/args.err
timeout -k 10 600 python -u -m pytest tests/test_graph_dp_gpu.py -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "FAILED|ERROR|Error" $O/tests.log | head -20
exit $rc
