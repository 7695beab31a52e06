#!/bin/bash
# Round-6 session 47: does a replayed hipGraph run the side-stream weight-gradient branch
# concurrently?  r6s46: eager + side stream 12,96-13,00k, graph + side stream = graph alone (12.84k).
# A/B of the HIP runtime's graph-queue knobs with DET_WGRAD_STREAM=1, plus eager side repeats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s47
mkdir -p $O
export TMPDIR=/tmp
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 60 --warmup 15 > $O/b.json 2> $O/b.err \
    || { echo "bench $tag rc=$?"; tail -20 $O/b.err; exit 1; }
  line=$(grep '^{' $O/b.json | tail -1)
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $O/ab.jsonl
  echo "$tag: $(echo "$line" | cut -c60-120)"
}
for rep in 1 2; do
  run graph_side DET_WGRAD_STREAM=1
  run graph_side_q2 DET_WGRAD_STREAM=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=2
  run graph_side_q4 DET_WGRAD_STREAM=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
  run graph_side_nopkt DET_WGRAD_STREAM=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run eager_side DET_WGRAD_STREAM=1 DET_HIP_GRAPH=0
done
