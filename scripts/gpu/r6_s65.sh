#!/bin/bash
# Round-6 session 65: default vs DET_NT_PF=2 + DET_STATS_FIRST=1 (the two most consistent small wins
# of r6s64), four alternating pairs at the default step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s65
mkdir -p $O
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 40 --warmup 10 > $O/b.json 2> $O/b.err \
    || { echo "bench $tag rc=$?"; tail -20 $O/b.err; exit 1; }
  line=$(grep '^{' $O/b.json | tail -1)
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $O/ab.jsonl
  echo "$tag: $(echo "$line" | grep -o '"value": [0-9.]*')"
}
for rep in 1 2 3 4; do
  run default DET_X=0
  run pf2_sf DET_NT_PF=2 DET_STATS_FIRST=1
done
