#!/bin/bash
# Round-6 session 62: the opt-in ResNet kernel knobs re-measured at the new default step (1,024
# images/GPU, eager + side stream): eight-phase wgrad (DET_WGRAD_CFG=14), igemm8 on 1x1 convs
# (DET_IGEMM8_1X1=1), bn2 in conv3's prologue (--bn-prologue).  Two alternating passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s62
mkdir -p $O
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 $EXTRA > $O/b.json 2> $O/b.err \
    || { echo "bench $tag rc=$?"; tail -20 $O/b.err; exit 1; }
  line=$(grep '^{' $O/b.json | tail -1)
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $O/ab.jsonl
  echo "$tag: $(echo "$line" | grep -o '"value": [0-9.]*')"
}
for rep in 1 2; do
  EXTRA="" run default DET_X=0
  EXTRA="" run wgrad8 DET_WGRAD_CFG=14
  EXTRA="" run igemm8_1x1 DET_IGEMM8_1X1=1
  EXTRA="--bn-prologue" run bn_prologue DET_X=0
done
