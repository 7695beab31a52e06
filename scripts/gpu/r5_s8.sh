#!/bin/bash
# Round-5 session 8: bisect the bf16 20-step-graph divergence of plain torch CIFAR steps (s7: replay 0
# exact, replay 1 diverges after eager steps ran in between; fp32 clean; every single op clean).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s8
mkdir -p $O
export TMPDIR=/tmp
R="python -u scripts/dbg/miopen_graph_repro.py --k 20"
for cfg in "noeager:--step --replays 6 --no-eager" "zero:--step --replays 5 --grads zero" "noupd:--step --replays 5 --update none" \
           "clob:--step --replays 4 --clobber 16" "noeager_clob:--step --replays 4 --no-eager --clobber 16" \
           "ops_clob:--replays 3 --clobber 8"; do
  name=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 300 $R $a > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "== $name"; grep -E '"mode"|"op"|"bad"' $O/$name.log | cut -c1-240
done
