#!/bin/bash
# Round-4 session 10: ASHA trials/hr on one GPU slot -- the r3 default (hip_graph_batches 20) vs the
# r2 configuration (1 batch per replay), and the reference precision (O0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s10
mkdir -p $O
export TMPDIR=/tmp
for cfg in "gb20:" "gb1:--graph-batches 1" "o0:--amp O0"; do
  name=${cfg%%:*}; args=${cfg#*:}
  DET_BENCH_LOGDIR=$O/asha_$name timeout -k 10 360 python -u scripts/bench_asha.py --slots 1 $args > $O/asha_$name.json 2> $O/asha_$name.err || { tail -30 $O/asha_$name.err; exit 1; }
  echo "asha $name $(cut -c1-300 $O/asha_$name.json)"
done
