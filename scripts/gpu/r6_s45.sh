#!/bin/bash
# Round-6 session 45: ASHA trials/hr at the reference adaptive.yaml shape on the round-6 tree (O0
# twice, O2 once), same command as round 5 (r5s37).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s45
mkdir -p $O
export TMPDIR=/tmp
for amp in O0 O0 O2; do
  DET_BENCH_LOGDIR=$O timeout -k 10 600 python -u scripts/bench_asha.py --slots 1 --amp $amp --graph-batches 20 --timeout 540 \
    > $O/asha.json 2> $O/asha.err || { echo "asha $amp rc=$?"; tail -20 $O/asha.err; exit 1; }
  grep '^{' $O/asha.json | tail -1 >> $O/asha_runs.jsonl
  echo "asha $amp: $(grep '^{' $O/asha.json | tail -1 | cut -c1-160)"
done
