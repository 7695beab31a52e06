#!/bin/bash
# Round-3 session 38 (fresh container, rebuilt .so): default bench on the rebuilt tree and attribution
# of the leftover copy/add/fill launches in the ResNet-50 step to their Python frames; full GPU tier + smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s38
mkdir -p $O
export TMPDIR=/tmp


timeout -k 10 400 python -u scripts/probe_small_launches.py --steps 3 --warmup 3 > $O/probe.txt 2> $O/probe.err || { tail -30 $O/probe.err; exit 1; }
grep -v '^{' $O/probe.txt | head -200
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
