#!/bin/bash
# Round-3 session 9: ASHA trials/hr at the BASELINE shape (16-trial adaptive_asha CIFAR-10, 32 epochs,
# validation every epoch, 1 slot) with 16-batch hipGraph replays, O2 and fp32/O0.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s9
mkdir -p $O
export TMPDIR=/tmp DET_BENCH_LOGDIR=$O
timeout -k 10 500 python -u scripts/bench_asha.py --slots 1 --timeout 450 > $O/asha_o2_gb16.json 2> $O/asha_o2_gb16.err || { tail -30 $O/asha_o2_gb16.err; exit 1; }
cat $O/asha_o2_gb16.json
cp $O/asha_timeline.txt $O/asha_o2_gb16_timeline.txt
timeout -k 10 600 python -u scripts/bench_asha.py --slots 1 --amp O0 --timeout 550 > $O/asha_o0_gb16.json 2> $O/asha_o0_gb16.err || { tail -30 $O/asha_o0_gb16.err; exit 1; }
cat $O/asha_o0_gb16.json
cp $O/asha_timeline.txt $O/asha_o0_gb16_timeline.txt
