#!/bin/bash
# Round-6 session 37: bench A/B of bn2 applied in conv3's GEMM prologue (--bn-prologue; a round-2
# negative result re-measured on the current kernels), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s37; mkdir -p $O
for i in 1 2; do
  for v in 1 0; do
    F=""; [ $v -eq 1 ] && F="--bn-prologue"
    timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 $F > $O/bench_pro$v.$i.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
    echo "prologue=$v: $(tail -1 $O/bench_pro$v.$i.json | python -c 'import sys,json; print(json.loads(sys.stdin.read())["value"])')"
  done
done
