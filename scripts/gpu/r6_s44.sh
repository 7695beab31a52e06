#!/bin/bash
# Round-6 session 44: 2,000 ResNet-50 steps eager vs hipGraph (memset rewrite on): parameters after
# the run compared (sums / norms per tensor), throughput of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s44; mkdir -p $O
for g in 0 1; do
  F=""; [ $g -eq 0 ] && F="--no-hip-graph"
  timeout -k 10 400 python -u bench.py --steps 2000 --warmup 5 $F --params-out $O/p$g.pt > $O/b$g.json 2> $O/b$g.err || { tail -20 $O/b$g.err; exit 1; }
  echo "graph=$g: $(tail -1 $O/b$g.json | cut -c1-160)"
done
python scripts/cmp_params.py $O/p0.pt $O/p1.pt --tol 1e-6 | tee $O/cmp.json
# the no-GradSink capture (DET_GRAPH_SINK=0) went non-finite before the memset rewrite (r6s12): again
DET_HIP_GRAPH=0 timeout -k 10 300 python -u scripts/dbg/graph_vs_eager_resnet.py --out $O/e.pt --steps 8 --bs 512 > $O/e.log 2>&1 || { tail $O/e.log; exit 1; }
DET_HIP_GRAPH=1 DET_GRAPH_SINK=0 timeout -k 10 300 python -u scripts/dbg/graph_vs_eager_resnet.py --out $O/gns.pt --steps 8 --bs 512 > $O/gns.log 2>&1 || { tail $O/gns.log; exit 1; }
python scripts/dbg/graph_vs_eager_resnet.py --compare $O/e.pt $O/gns.pt | tail -4
