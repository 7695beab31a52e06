#!/bin/bash
# Round-5 session 1: the O2 hipGraph + dropout NaN.  Per-replay invariants (bf16 arena == bf16(master),
# zero grad arena, intact static inputs, finite loss/masters) with stock torch dropout, a torch.rand
# mask, and a fixed mask bank (no RNG kernel in the graph); eager control.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s1
mkdir -p $O
export TMPDIR=/tmp
for cfg in "torch_g1:--variant torch" "bank_g1:--variant bankmask" "rand_g1:--variant randmask" "torch_eager:--variant torch --no-graph"; do
  name=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 240 python -u scripts/dbg/graph_nan_probe.py $a --batches 2200 --out $O > $O/$name.json 2> $O/$name.err \
    || { echo "$name failed rc=$?"; tail -30 $O/$name.err; exit 1; }
  echo "== $name"; cat $O/$name.json
done
