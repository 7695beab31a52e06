#!/bin/bash
# Round-5 session 10: which library diverges in the bf16 20-step graph with grads set to None and
# eager steps between replays (s8/s9): convolutions only, linears only, MIOpen off, rocBLAS for GEMMs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s10
mkdir -p $O
export TMPDIR=/tmp
R="python -u scripts/dbg/miopen_graph_repro.py --k 20 --step --replays 4"
for cfg in "conv:--arch conv" "mlp:--arch mlp" "nomiopen:--no-miopen" "conv_nomiopen:--arch conv --no-miopen"; do
  name=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 300 $R $a > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "== $name"; grep -E '"mode"' $O/$name.log | cut -c1-200
done
TORCH_BLAS_PREFER_HIPBLASLT=0 timeout -k 10 300 $R > $O/rocblas.log 2>&1 || { echo "rocblas rc=$?"; tail -20 $O/rocblas.log; exit 1; }
echo "== rocblas"; grep -E '"mode"' $O/rocblas.log | cut -c1-200
TORCH_BLAS_PREFER_HIPBLASLT=0 timeout -k 10 300 $R --arch mlp > $O/mlp_rocblas.log 2>&1 || { echo "mlp_rocblas rc=$?"; tail -20 $O/mlp_rocblas.log; exit 1; }
echo "== mlp rocblas"; grep -E '"mode"' $O/mlp_rocblas.log | cut -c1-200
