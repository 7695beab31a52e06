#!/bin/bash
# Round-3 session 38 (fresh container, rebuilt .so): default bench on the rebuilt tree and attribution
# of the leftover copy/add/fill launches in the ResNet-50 step to their Python frames.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s38
mkdir -p $O
export TMPDIR=/tmp


timeout -k 10 400 python -u scripts/probe_small_launches.py --steps 3 --warmup 3 > $O/probe.txt 2> $O/probe.err || { tail -30 $O/probe.err; exit 1; }
grep -v '^{' $O/probe.txt | head -200
