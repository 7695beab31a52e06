#!/bin/bash
# Round-5 session 27: per-kernel split of the LayerNorm forward / backward at the BERT shape
# (rocprofv3 kernel stats), default and narrow forward.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s27
mkdir -p $O
export TMPDIR=/tmp
for f in wide narrow; do
  DET_LN_FWD=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lnprof_$f -o ln -- python3 -u scripts/bench_ln.py --iters 200 > $O/ln_$f.json 2> $O/ln.err || { tail -20 $O/ln.err; exit 1; }
  cat $O/ln_$f.json
  find /tmp/lnprof_$f -name "*kernel_stats.csv" -exec cp {} $O/ln_${f}_kernel_stats.csv \;
  python3 -c "
import csv
rows=list(csv.DictReader(open('$O/ln_${f}_kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')
"
done
