#!/bin/bash
# Round-6 session 64: kernel-variant knobs re-measured at the new default step (1,024 images/GPU,
# eager + side stream, wgrad8): each knob against the default, two alternating passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s64
mkdir -p $O
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/b.json 2> $O/b.err \
    || { echo "bench $tag rc=$?"; tail -20 $O/b.err; exit 1; }
  line=$(grep '^{' $O/b.json | tail -1)
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $O/ab.jsonl
  echo "$tag: $(echo "$line" | grep -o '"value": [0-9.]*')"
}
for rep in 1 2; do
  run default DET_X=0
  run wgrad_wgs256 DET_WGRAD_WGS=256
  run wgrad_wgs1024 DET_WGRAD_WGS=1024
  run nt_pf2 DET_NT_PF=2
  run bnb_pf2 DET_BNB_PF=2
  run nt_wide DET_NT_WIDE=1
  run stats_first DET_STATS_FIRST=1
  run bnb_occ2 DET_BNB_SINGLE_OCC=0
  run conv3p_wgrad_off DET_CONV3P_WGRAD=0
done
