#!/bin/bash
# Round-2 session 24: does the MI355X run several small trials concurrently?  1, 2, 4 and 8
# simultaneous CIFAR trial processes (hipGraph, batch 32) on one GPU: aggregate records/s.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s24
export TMPDIR=/tmp
for n in 1 2 4 8; do
  pids=()
  for i in $(seq 1 $n); do
    timeout -k 10 200 python -u scripts/bench_cifar_trial.py --batch 32 --batches 3000 --hip-graph > gpurun_out/s24/n${n}_$i.json 2> gpurun_out/s24/n${n}_$i.err &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait $p || { echo "run failed (n=$n)"; tail -5 gpurun_out/s24/n${n}_*.err; exit 1; }; done
  python - "$n" <<'PY'
import json, sys, glob
n = int(sys.argv[1])
rs = [json.load(open(f)) for f in sorted(glob.glob(f"gpurun_out/s24/n{n}_*.json"))]
print(json.dumps({"concurrent_trials": n, "ms_per_batch_each": [r["value"] for r in rs],
                  "aggregate_records_per_s": round(sum(r["records_per_s"] for r in rs), 1)}))
PY
done
