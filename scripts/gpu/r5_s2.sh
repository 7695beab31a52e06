#!/bin/bash
# Round-5 session 2: (a) the O2 hipGraph + dropout NaN probe (guard lifted inside the probe);
# (b) HBM streaming yardstick sweep + FETCH_SIZE/WRITE_SIZE calibration on known byte counts.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s2
mkdir -p $O
export TMPDIR=/tmp
for cfg in "torch_g1:--variant torch" "bank_g1:--variant bankmask" "rand_g1:--variant randmask" "torch_eager:--variant torch --no-graph"; do
  name=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 240 python -u scripts/dbg/graph_nan_probe.py $a --batches 2200 --out $O > $O/$name.json 2> $O/$name.err \
    || { echo "$name failed rc=$?"; tail -30 $O/$name.err; exit 1; }
  echo "== $name"; cat $O/$name.json
done
timeout -k 10 300 python -u scripts/bench_stream.py --sweep --out $O/stream_sweep.jsonl > $O/stream_best.jsonl 2> $O/stream.err \
  || { echo "stream sweep failed"; tail -20 $O/stream.err; exit 1; }
cat $O/stream_best.jsonl
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_$c -o run --output-format csv -- python3 scripts/bench_stream.py --calib --max-gib 2 \
    > $O/calib_$c.log 2>&1 || { echo "calib $c failed"; tail -20 $O/calib_$c.log; exit 1; }
done
find $O -name "*counter_collection.csv" | head
