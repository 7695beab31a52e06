#!/bin/bash
# Round-6 session 32: steady-state kernel profile of the current ResNet-50 bench step (hipGraph,
# igemm8 defaults), the summary committed as profiles/r6_resnet50_steady.{txt,csv}.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s32; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o resnet --output-format csv -- python3 bench.py --steps 30 --warmup 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "resnet_kernel_trace.csv" | head -1)
python scripts/prof_summarize.py $f --skip-steps 8 --out $O/steady.csv > $O/steady.txt 2>&1; rc=$?
head -45 $O/steady.txt
exit $rc
