#!/bin/bash
# Round-3 session 1: det_igemm v2 (software-pipelined fragment reads) tile configs vs v1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3s1
export TMPDIR=/tmp
timeout -k 10 400 ./scripts/kbench/igemm_bench 512 1,2,8,11 1 > gpurun_out/r3s1/igemm_cfgs.jsonl 2> gpurun_out/r3s1/igemm_cfgs.err
rc=$?
tail -5 gpurun_out/r3s1/igemm_cfgs.err
exit $rc
