#!/bin/bash
# Round-6 session 22: ResNet-50 data-parallel steps (world-1 RCCL group, DET_FORCE_DISTRIBUTED) under
# hipGraph after the captured-memset rewrite: graph vs eager parameters after 100 steps, and a kernel
# trace of the graph run (RCCL kernels inside the replays).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s22
mkdir -p $O
export TMPDIR=/tmp WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 DET_FORCE_DISTRIBUTED=1
p=29670
for g in 0 1; do
  p=$((p+1))
  MASTER_PORT=$p DET_HIP_GRAPH=$g timeout -k 10 400 python -u bench.py --steps 100 --warmup 5 --params-out $O/resnet_g$g.pt > $O/resnet_g$g.json 2> $O/resnet_g$g.err || { tail -20 $O/resnet_g$g.err; exit 1; }
  echo "resnet dp graph=$g: $(cut -c1-200 $O/resnet_g$g.json)"
done
python scripts/cmp_params.py $O/resnet_g0.pt $O/resnet_g1.pt --tol 1e-3 | tee $O/resnet_cmp.json
p=$((p+1))
MASTER_PORT=$p DET_HIP_GRAPH=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o resnet_dpg --output-format csv -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "resnet_dpg_kernel_stats.csv" | head -1); grep -i -E "nccl|rccl" $f | cut -c1-200 | head
