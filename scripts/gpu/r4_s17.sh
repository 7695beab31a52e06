#!/bin/bash
# Round-4 session 17: where the ASHA trial's time goes (CIFAR-10 trial through the controller, the
# adaptive.yaml configuration: O2, hipGraph replays of 20-batch chunks): ms/batch and validation,
# then a kernel trace of the same run (kernel-busy fraction of the steady window).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s17
mkdir -p $O
export TMPDIR=/tmp
for b in 32 64; do
  timeout -k 10 300 python -u scripts/bench_cifar_trial.py --batch $b --batches 3000 --hip-graph --graph-batches 20 > $O/cifar_b$b.json 2> $O/cifar_b$b.err || { tail -30 $O/cifar_b$b.err; exit 1; }
  echo "cifar b$b $(cut -c1-400 $O/cifar_b$b.json)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u scripts/bench_cifar_trial.py --batch 32 --batches 1500 --hip-graph --graph-batches 20 > $O/cifar_prof.json 2> $O/cifar_prof.err || { tail -20 $O/cifar_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summarize.py "$f" --out $O/cifar_steady.csv > $O/cifar_steady.txt 2>&1 || { tail -5 $O/cifar_steady.txt; exit 1; }
head -25 $O/cifar_steady.txt
rm -rf $O/prof
