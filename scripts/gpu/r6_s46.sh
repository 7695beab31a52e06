#!/bin/bash
# Round-6 session 46: conv weight gradients on a side stream (DET_WGRAD_STREAM=1).  Parity test
# (eager + graph), then ResNet-50 bench A/B, alternating order, eager and graph.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s46
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_wgrad_stream_gpu.py \
  > $O/test.log 2>&1 || { echo "test rc=$?"; tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
for rep in 1 2; do
  for side in 0 1; do
    for graph in 1 0; do
      flag=""; [ $graph = 0 ] && flag="--no-hip-graph"
      DET_WGRAD_STREAM=$side timeout -k 10 300 python -u bench.py --steps 60 --warmup 15 $flag > $O/b.json 2> $O/b.err \
        || { echo "bench side=$side graph=$graph rc=$?"; tail -20 $O/b.err; exit 1; }
      line=$(grep '^{' $O/b.json | tail -1)
      echo "{\"side\": $side, \"graph\": $graph, \"rep\": $rep, \"bench\": $line}" >> $O/ab.jsonl
      echo "side=$side graph=$graph rep=$rep: $(echo "$line" | cut -c1-110)"
    done
  done
done
