#!/bin/bash
# Round-6 session 5: which RCCL collectives capture into a hipGraph (world 1), with and without the
# process-group watchdog.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s5
mkdir -p $O
export TMPDIR=/tmp
NCCL_DEBUG=WARN timeout -k 10 400 python -u scripts/dbg/rccl_capture.py > $O/capture.jsonl 2> $O/capture.err
rc=$?; echo "rc=$rc"; cat $O/capture.jsonl | cut -c1-400
[ $rc -eq 0 ] || exit $rc
TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0 NCCL_DEBUG=WARN timeout -k 10 400 python -u scripts/dbg/rccl_capture.py > $O/capture_nowd.jsonl 2> $O/capture_nowd.err
rc=$?; echo "nowd rc=$rc"; cat $O/capture_nowd.jsonl | cut -c1-400
exit $rc
