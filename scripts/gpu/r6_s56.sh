#!/bin/bash
# Round-6 session 56: BERT-base SQuAD shape, hipGraph replay, HIP_FORCE_DEV_KERNARG=0 vs 1 (kernel
# arguments in device memory; measured only on eager BERT before, where it loses).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s56
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in 0 1; do
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python -u scripts/bench_bert.py --steps 200 --warmup 10 --hip-graph \
      > $O/b.json 2> $O/b.err || { echo "bert kernarg=$v rc=$?"; tail -20 $O/b.err; exit 1; }
    line=$(grep '^{' $O/b.json | tail -1)
    echo "{\"dev_kernarg\": $v, \"bench\": $line}" >> $O/ab.jsonl
    echo "kernarg=$v: $(echo "$line" | cut -c80-135)"
  done
done
