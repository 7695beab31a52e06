#!/bin/bash
# Round-6 session 35: bench A/B/C: igemm8 off / 3x3 only / 3x3 + selected 1x1, three rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s35; mkdir -p $O
for i in 1 2 3; do
  for v in off r3 all; do
    case $v in off) E="DET_IGEMM8=0";; r3) E="DET_IGEMM8_1X1=0";; all) E="DET_IGEMM8=1";; esac
    env $E timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 > $O/bench_$v.$i.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
    echo "$v: $(tail -1 $O/bench_$v.$i.json | cut -c80-120)"
  done
done
