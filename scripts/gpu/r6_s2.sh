#!/bin/bash
# Round-6 session 2: per-key graph probe GPU tests, and the node census of captured library convs
# (what a captured MIOpen conv1_bwd_weight puts in the graph).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/dbg/graph_nodes.py --dtype bf16 > $O/nodes_bf16.jsonl 2> $O/nodes.err; echo "nodes rc=$?"
timeout -k 10 300 python -u scripts/dbg/graph_nodes.py --dtype fp32 > $O/nodes_fp32.jsonl 2>> $O/nodes.err; echo "nodes fp32 rc=$?"
cut -c1-300 $O/nodes_bf16.jsonl; tail -5 $O/nodes.err
timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py tests/test_graph_cifar_o2_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -20
exit $rc
